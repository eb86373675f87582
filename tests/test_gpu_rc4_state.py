"""rc4.h on the device: ``ops.rc4_crypt_batch`` continues many ``struct
rc4_state`` streams (reference rc4.h:43-50) in one launch and writes every
state back, so split calls equal one host ``rc4_crypt`` per stream (SURVEY
2.2 C5: "routed to the same HIP RC4 kernels")."""
import ctypes
import os

import pytest
import torch

from our_tree_amd import _native, ops


def _host_rc4(key: bytes, chunks):
    lib = _native.cpu_lib()
    st = _native.Rc4State()
    lib.rc4_init(ctypes.byref(st), key, len(key))
    outs = []
    for c in chunks:
        o = ctypes.create_string_buffer(len(c))
        lib.rc4_crypt(ctypes.byref(st), c, o, len(c))
        outs.append(o.raw)
    return outs, bytes(st)


def test_rc4_state_images_match_struct():
    keys = [b"Key", os.urandom(16)]
    t = ops.rc4_states(keys)
    assert t.shape == (2, 264)
    for k, row in zip(keys, t):
        _, st = _host_rc4(k, [])
        assert bytes(row.numpy().tobytes()) == st


@pytest.mark.gpu
@pytest.mark.parametrize("l1,l2", [(37, 64), (64, 4096 + 5), (1, 1)])
def test_rc4_crypt_batch_resumes_like_host(gpu, l1, l2):
    n = 300  # not a multiple of the 64-lane workgroup
    keys = [os.urandom(1 + (r % 32)) for r in range(n)]
    states = ops.rc4_states(keys).to(gpu)
    a = torch.randint(0, 256, (n, l1), dtype=torch.uint8, device=gpu)
    b = torch.randint(0, 256, (n, l2), dtype=torch.uint8, device=gpu)
    ya = ops.rc4_crypt_batch(states, a)
    yb = ops.rc4_crypt_batch(states, b, out=b.clone())
    torch.cuda.synchronize()
    ya, yb, sa, sb, st = ya.cpu(), yb.cpu(), a.cpu(), b.cpu(), states.cpu()
    for r in (0, 1, 63, 64, 127, 255, 299):
        (ea, eb), est = _host_rc4(keys[r], [sa[r].numpy().tobytes(), sb[r].numpy().tobytes()])
        assert ya[r].numpy().tobytes() == ea, r
        assert yb[r].numpy().tobytes() == eb, r
        assert st[r].numpy().tobytes() == est, r  # state written back (perm, index1, index2)


@pytest.mark.gpu
def test_rc4_crypt_batch_in_place_and_validation(gpu):
    keys = [b"Secret", b"Key"]
    states = ops.rc4_states(keys).to(gpu)
    x = torch.randint(0, 256, (2, 1000), dtype=torch.uint8, device=gpu)
    src = x.cpu()
    ops.rc4_crypt_batch(states, x, out=x)
    torch.cuda.synchronize()
    for r in range(2):
        (e,), _ = _host_rc4(keys[r], [src[r].numpy().tobytes()])
        assert x[r].cpu().numpy().tobytes() == e
    with pytest.raises(ValueError):
        ops.rc4_crypt_batch(states[:, :200].contiguous(), x)
    with pytest.raises(ValueError):
        ops.rc4_crypt_batch(states, torch.zeros(3, device=gpu, dtype=torch.uint8))
