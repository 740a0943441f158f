"""TEST INFRASTRUCTURE ONLY -- the reference's server loop, restated line for line in numpy.

This is the CPU baseline that bench.py times beside the GPU (kind "port").
It follows the reference's own statements and their cost structure:
  vec_sum_partial = zeros; vec_sum_partial += user_vectors[id]      SA_ServiceAgent.py:346-350
  mi_vec = mi_vec - np.frombuffer(ChaCha20(m_i).encrypt(b"abcd"*L))  :530-536
  cancel_vec = cancel_vec +/- np.frombuffer(ChaCha20(s_ij)...)       :595-603
  final_sum = vec_sum_partial + cancel_vec + mi_vec                  :605
The cipher in the reference is pycryptodomex's C ChaCha20 (not installed
here); this restatement calls OpenSSL's C ChaCha20 (EVP_chacha20, zero IV ==
the 8-byte zero nonce DJB stream) through ctypes.  It is checked against
the C oracle and the GPU result, and the C oracle against the reference's own
rounds (tests/test_ref_golden_cpu.py).  Single-threaded, like the reference server.
"""
from __future__ import annotations

import ctypes

import numpy as np

_crypto = None


def _lib():
    global _crypto
    if _crypto is None:
        c = ctypes.CDLL("libcrypto.so.3")
        c.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        c.EVP_chacha20.restype = ctypes.c_void_p
        c.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                         ctypes.c_char_p]
        c.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                        ctypes.c_void_p, ctypes.c_int]
        c.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        _crypto = c
    return _crypto


def chacha20_encrypt(key: bytes, data: bytes) -> bytes:
    """ChaCha20.new(key=key, nonce=8x00).encrypt(data) via OpenSSL."""
    c = _lib()
    ctx = c.EVP_CIPHER_CTX_new()
    try:
        assert c.EVP_EncryptInit_ex(ctx, c.EVP_chacha20(), None, key, b"\x00" * 16) == 1
        out = ctypes.create_string_buffer(len(data))
        n = ctypes.c_int(0)
        assert c.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), data, len(data)) == 1
        return out.raw
    finally:
        c.EVP_CIPHER_CTX_free(ctx)


def server_round(user_vectors, mi_seeds, pair_seeds, recon_symbols, L: int) -> np.ndarray:
    """The reference's report_process sum + reconstruction_process unmask, as written there."""
    fixed_key = b"abcd"
    vec_sum_partial = np.zeros(L, dtype="uint32")
    for v in user_vectors:
        if len(v) != L:
            raise RuntimeError("Client sends vector of incorrect length.")
        vec_sum_partial += v
    mi_vec = np.zeros(L, dtype="uint32")
    for s in mi_seeds:
        prg = chacha20_encrypt(s, fixed_key * L)
        mi_vec = mi_vec - np.frombuffer(prg, dtype="uint32")
    if not pair_seeds:
        return vec_sum_partial + mi_vec
    cancel_vec = np.zeros(L, dtype="uint32")
    for s, sym in zip(pair_seeds, recon_symbols):
        prg = chacha20_encrypt(s, fixed_key * L)
        if sym == 1:
            cancel_vec = cancel_vec + np.frombuffer(prg, dtype="uint32")
        elif sym == -1:
            cancel_vec = cancel_vec - np.frombuffer(prg, dtype="uint32")
    return vec_sum_partial + cancel_vec + mi_vec
