/*
 * otc_numa.h -- host NUMA placement helpers (csrc/cpu/numa.c).
 *
 * Used by the streaming engine / multi-GPU direct ingest to put each GPU's
 * pinned staging window and host worker thread on the GPU's socket.
 * `sysfs_root` = NULL means "/sys" (tests pass a fake tree).
 */
#ifndef OTC_NUMA_H
#define OTC_NUMA_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OTC_NUMA_MAXCPU 4096

/* Linux cpulist syntax ("0-23,48-71", "0-31:2") -> mask[cpu] = 1.
 * Returns the number of CPUs set, -1 on a syntax error. */
int otc_parse_cpulist(const char *s, unsigned char *mask, int maxcpu);
/* NUMA node of a PCI device ("0000:05:00.0"), -1 if unknown. */
int otc_numa_node_of_pci(const char *sysfs_root, const char *pci_bus_id);
/* CPUs of `node` into mask; returns their count or -1. */
int otc_numa_node_cpus(const char *sysfs_root, int node, unsigned char *mask, int maxcpu);
/* Number of online NUMA nodes (>= 1). */
int otc_numa_num_nodes(const char *sysfs_root);
/* Pin the calling thread to the CPUs of `node` that its cpuset allows;
 * returns how many (0 for node < 0, -1 if none / failure: affinity unchanged). */
int otc_numa_bind_thread(int node);
/* Page-aligned anonymous memory placed on `node` (preferred), pre-faulted. */
void *otc_numa_alloc(size_t nbytes, int node);
void otc_numa_free(void *p, size_t nbytes);
/* Node holding the page at `p` (-1 if unknown). */
int otc_numa_node_of_addr(const void *p);

#ifdef __cplusplus
}
#endif

#endif
