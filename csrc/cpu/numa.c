/*
 * numa.c -- NUMA placement for host ingest (no libnuma: sysfs + raw syscalls).
 *
 * On an 8-GPU MI355X node the GPUs hang off two CPU sockets; a GPU's pinned
 * staging window should live in the DRAM of the socket its PCIe root port is
 * on, and the host thread that fills it should run on that socket's cores
 * (SURVEY.md 7.4 item 5).  The reference had no host placement at all (its
 * only host path was synchronous pageable copies, aes-gpu/Source/AES.cu:236,252).
 *
 * Every sysfs lookup takes the sysfs root as a parameter so the placement
 * logic is unit-tested on the CPU against a fake tree (tests/test_numa_cpu.py).
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <errno.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "otc_numa.h"

#ifndef MPOL_DEFAULT
#define MPOL_DEFAULT 0
#define MPOL_PREFERRED 1
#define MPOL_BIND 2
#endif
#ifndef MPOL_F_NODE
#define MPOL_F_NODE (1 << 0)
#define MPOL_F_ADDR (1 << 1)
#endif

static const char *root_or_default(const char *sysfs_root) { return sysfs_root && *sysfs_root ? sysfs_root : "/sys"; }

static int read_small(const char *path, char *buf, size_t cap)
{
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    size_t n = fread(buf, 1, cap - 1, f);
    fclose(f);
    buf[n] = 0;
    while (n && isspace((unsigned char)buf[n - 1])) buf[--n] = 0;
    return (int)n;
}

int otc_parse_cpulist(const char *s, unsigned char *mask, int maxcpu)
{
    if (!s || !mask || maxcpu <= 0) return -1;
    memset(mask, 0, (size_t)maxcpu);
    int count = 0;
    const char *p = s;
    while (*p) {
        while (*p == ',' || isspace((unsigned char)*p)) ++p;
        if (!*p) break;
        if (!isdigit((unsigned char)*p)) return -1;
        char *end;
        long a = strtol(p, &end, 10), b = a, step = 1;
        p = end;
        if (*p == '-') {
            ++p;
            if (!isdigit((unsigned char)*p)) return -1;
            b = strtol(p, &end, 10);
            p = end;
            if (*p == ':') { /* "0-31:2" stride form */
                ++p;
                step = strtol(p, &end, 10);
                p = end;
                if (step < 1) return -1;
            }
        }
        if (b < a || a < 0) return -1;
        for (long c = a; c <= b; c += step)
            if (c < maxcpu && !mask[c]) {
                mask[c] = 1;
                ++count;
            }
        if (*p && *p != ',' && !isspace((unsigned char)*p)) return -1;
    }
    return count;
}

int otc_numa_node_of_pci(const char *sysfs_root, const char *pci_bus_id)
{
    if (!pci_bus_id || !*pci_bus_id) return -1;
    char id[64];
    size_t n = strlen(pci_bus_id);
    if (n >= sizeof id) return -1;
    for (size_t i = 0; i <= n; ++i) id[i] = (char)tolower((unsigned char)pci_bus_id[i]);
    char path[512], buf[32];
    snprintf(path, sizeof path, "%s/bus/pci/devices/%s/numa_node", root_or_default(sysfs_root), id);
    if (read_small(path, buf, sizeof buf) <= 0) return -1;
    int node = atoi(buf);
    return node >= 0 ? node : -1; /* -1 in sysfs = no NUMA information */
}

int otc_numa_node_cpus(const char *sysfs_root, int node, unsigned char *mask, int maxcpu)
{
    if (node < 0) return -1;
    char path[512], buf[4096];
    snprintf(path, sizeof path, "%s/devices/system/node/node%d/cpulist", root_or_default(sysfs_root), node);
    if (read_small(path, buf, sizeof buf) < 0) return -1;
    return otc_parse_cpulist(buf, mask, maxcpu);
}

int otc_numa_num_nodes(const char *sysfs_root)
{
    char path[512], buf[256];
    snprintf(path, sizeof path, "%s/devices/system/node/online", root_or_default(sysfs_root));
    if (read_small(path, buf, sizeof buf) <= 0) return 1;
    unsigned char mask[1024];
    int c = otc_parse_cpulist(buf, mask, 1024); /* same range syntax */
    return c > 0 ? c : 1;
}

int otc_numa_bind_thread(int node)
{
    if (node < 0) return 0;
    unsigned char mask[OTC_NUMA_MAXCPU];
    int c = otc_numa_node_cpus(NULL, node, mask, OTC_NUMA_MAXCPU);
    if (c <= 0) return -1;
    cpu_set_t set;
    CPU_ZERO(&set);
    int allowed = 0;
    cpu_set_t cur;
    CPU_ZERO(&cur);
    if (sched_getaffinity(0, sizeof cur, &cur) != 0) return -1;
    for (int i = 0; i < OTC_NUMA_MAXCPU && i < CPU_SETSIZE; ++i)
        if (mask[i] && CPU_ISSET(i, &cur)) {
            CPU_SET(i, &set);
            ++allowed;
        }
    if (!allowed) return -1; /* the node's CPUs are outside our cpuset: leave it */
    return sched_setaffinity(0, sizeof set, &set) == 0 ? allowed : -1;
}

/* Anonymous mapping whose pages are bound to `node` (mbind before first
 * touch, then touched so they are resident there).  node < 0: plain mapping. */
void *otc_numa_alloc(size_t nbytes, int node)
{
    if (nbytes == 0) return NULL;
    void *p = mmap(NULL, nbytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return NULL;
    if (node >= 0 && node < 64) {
        unsigned long nodemask = 1ul << node;
        /* MPOL_PREFERRED: placed on `node` while it has free memory, never a
         * hard failure */
        (void)syscall(SYS_mbind, p, nbytes, MPOL_PREFERRED, &nodemask, 64ul, 0u);
    }
    const long pg = sysconf(_SC_PAGESIZE);
    for (size_t o = 0; o < nbytes; o += (size_t)(pg > 0 ? pg : 4096)) ((volatile char *)p)[o] = 0;
    return p;
}

void otc_numa_free(void *p, size_t nbytes)
{
    if (p && nbytes) munmap(p, nbytes);
}

int otc_numa_node_of_addr(const void *p)
{
    int node = -1;
    if (syscall(SYS_get_mempolicy, &node, NULL, 0ul, (void *)p, MPOL_F_NODE | MPOL_F_ADDR) != 0) return -1;
    return node;
}
