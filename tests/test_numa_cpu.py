"""NUMA placement helpers (csrc/cpu/numa.c) against a fake sysfs tree: the
logic that puts each GPU's pinned staging ring and host worker thread on the
GPU's socket is unit-tested without a GPU or a multi-socket machine."""
import ctypes

import pytest

from our_tree_amd import _native


@pytest.fixture(scope="module")
def lib():
    return _native.cpu_lib()


def _mask(lib, s, maxcpu=256):
    m = (ctypes.c_uint8 * maxcpu)()
    n = lib.otc_parse_cpulist(s.encode(), m, maxcpu)
    return n, [i for i in range(maxcpu) if m[i]]


@pytest.mark.parametrize("s,cpus", [
    ("0", [0]),
    ("0-3", [0, 1, 2, 3]),
    ("0-1,8-9", [0, 1, 8, 9]),
    ("0-7:2", [0, 2, 4, 6]),
    ("2,0,2", [0, 2]),
    ("", []),
    ("0-3\n", [0, 1, 2, 3]),
])
def test_parse_cpulist(lib, s, cpus):
    n, got = _mask(lib, s)
    assert n == len(cpus) and got == cpus


@pytest.mark.parametrize("bad", ["a", "3-1", "1-", "1-2x", "-1"])
def test_parse_cpulist_rejects(lib, bad):
    assert _mask(lib, bad)[0] == -1


def _fake_sysfs(tmp_path, gpus, nodes):
    for bus, node in gpus.items():
        d = tmp_path / "bus" / "pci" / "devices" / bus
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
    for node, cpulist in nodes.items():
        d = tmp_path / "devices" / "system" / "node" / f"node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpulist + "\n")
    (tmp_path / "devices" / "system" / "node" / "online").write_text(
        ",".join(str(n) for n in sorted(nodes)) + "\n")
    return str(tmp_path).encode()


def test_gpu_to_node_to_cpus(lib, tmp_path):
    # 8 GPUs on 2 sockets, the typical MI355X node layout
    gpus = {f"0000:{b:02x}:00.0": (0 if i < 4 else 1) for i, b in enumerate((0x05, 0x15, 0x65, 0x75, 0x85, 0x95,
                                                                             0xe5, 0xf5))}
    root = _fake_sysfs(tmp_path, gpus, {0: "0-63,128-191", 1: "64-127,192-255"})
    assert lib.otc_numa_num_nodes(root) == 2
    for bus, node in gpus.items():
        assert lib.otc_numa_node_of_pci(root, bus.upper().encode()) == node  # HIP reports upper-case hex
    m = (ctypes.c_uint8 * 512)()
    assert lib.otc_numa_node_cpus(root, 1, m, 512) == 128
    assert m[64] and m[255] and not m[0] and not m[128]


def test_unknown_placement(lib, tmp_path):
    root = _fake_sysfs(tmp_path, {"0000:05:00.0": -1}, {0: "0-7"})
    assert lib.otc_numa_node_of_pci(root, b"0000:05:00.0") == -1   # sysfs -1: no NUMA info
    assert lib.otc_numa_node_of_pci(root, b"0000:99:00.0") == -1   # no such device
    m = (ctypes.c_uint8 * 64)()
    assert lib.otc_numa_node_cpus(root, 3, m, 64) == -1
    assert lib.otc_numa_bind_thread(-1) == 0                       # unknown node: leave affinity alone


def test_numa_alloc_on_this_machine(lib):
    n = 1 << 20
    p = lib.otc_numa_alloc(n, 0)
    assert p
    ctypes.memset(p, 0xAB, n)
    node = lib.otc_numa_node_of_addr(p)
    assert node in (-1, 0)   # -1 if the container forbids get_mempolicy
    lib.otc_numa_free(p, n)
