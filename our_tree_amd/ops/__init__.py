"""Device ops (gfx950 HIP kernels) on torch tensors."""
from .aes_ops import (IMPLS, CtrBatch, CtrStream, cbc_decrypt, cbc_decrypt_segments, cbc_encrypt_segments, cfb128_decrypt,
                      cfb128_decrypt_segments, cfb128_encrypt_segments,
                      ctr, ctr_batch, ctr_rfc3686, ecb_decrypt, ecb_encrypt, last_impl, pick_impl,
                      split_fallback_reason)
from .keys import expand_key
from .stream_ops import checksum, clock_ghz, clock_probe, fill_random_, rc4_crypt_batch, rc4_multi, rc4_states, xor

__all__ = [
    "IMPLS", "ctr", "ctr_batch", "CtrBatch", "CtrStream", "ctr_rfc3686", "ecb_encrypt", "ecb_decrypt", "cbc_decrypt", "cbc_encrypt_segments",
    "cbc_decrypt_segments", "cfb128_decrypt", "cfb128_encrypt_segments", "cfb128_decrypt_segments", "expand_key", "xor", "rc4_multi", "fill_random_", "checksum",
    "clock_probe", "clock_ghz", "pick_impl", "last_impl", "split_fallback_reason", "rc4_states", "rc4_crypt_batch",
]
