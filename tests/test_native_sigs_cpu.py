"""Every native function the Python side calls has a declared ctypes
signature (our_tree_amd/_native.py).  An undeclared one gets ctypes'
defaults -- int arguments and result -- so a 64-bit pointer is truncated to
32 bits: otc_ptr_kind ran that way through round 4 and classified every
pinned buffer as pageable (the RCCL job's "pageable" warning fired for
pinned_empty() buffers)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _py_files():
    for top in ("our_tree_amd", "tests", "benchmarks", "tools"):
        for d, _, fs in os.walk(os.path.join(ROOT, top)):
            for f in fs:
                if f.endswith(".py"):
                    yield os.path.join(d, f)
    for f in ("bench.py", "__graft_entry__.py"):
        yield os.path.join(ROOT, f)


def test_every_called_native_function_is_declared():
    declared = set(re.findall(r'"(otc_\w+)": \(', open(os.path.join(ROOT, "our_tree_amd", "_native.py")).read()))
    used = set()
    for p in _py_files():
        if os.path.exists(p) and os.path.basename(p) != os.path.basename(__file__):
            used |= set(re.findall(r"\.(otc_\w+)\(", open(p).read()))
    assert used, "no native calls found"
    assert used <= declared, sorted(used - declared)


def test_pointer_arguments_are_pointer_typed():
    """otc_ptr_kind takes a void pointer (not the int default)."""
    src = open(os.path.join(ROOT, "our_tree_amd", "_native.py")).read()
    assert re.search(r'"otc_ptr_kind": \(c_int, \[c_vp\]\)', src)
