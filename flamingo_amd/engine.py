"""Host-side handle on the MI355X engine (libflamingo_hip.so).

``MaskEngine`` owns one C-ABI context bound to one GPU (one process per GPU).
Its methods are the calls the drop-in agents make in place of the reference's
numpy/pycryptodomex loops:

* ``aggregate_unmask`` -- SA_ServiceAgent.report_process partial sum
  (agent/flamingo/SA_ServiceAgent.py:346-350) + reconstruction_process unmask
  and combine (:529-540, :587-605).
* ``client_mask`` -- SA_ClientAgent.sendVectors mask composition
  (agent/flamingo/SA_ClientAgent.py:246-324), batched over clients.
* ``prg_expand`` / ``prg`` -- the PRG idiom ChaCha20(seed).encrypt(b"abcd"*L)
  viewed as uint32 (SA_ClientAgent.py:248-250).
* ``chacha20_encrypt`` -- ChaCha20.new(key, nonce).encrypt(data) for the
  PRF/PRG calls of util/param.py:44-46, 63-76.
* ``*_dev`` -- the same on device-resident torch tensors (bench, multi-GPU).

Errors surface as RuntimeError with the library's message, like the
reference's own guards (SA_ServiceAgent.py:349, 502).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import p_i8, p_i64, p_u8, p_u32

NONCE = b"\x00" * 8


def _seeds_array(seeds) -> np.ndarray:
    if isinstance(seeds, (list, tuple)):
        if len(seeds) == 0:
            return np.zeros((0, 32), np.uint8)
        if isinstance(seeds[0], (bytes, bytearray)):
            if any(len(s) != 32 for s in seeds):
                raise RuntimeError("every seed must be 32 bytes")
            return np.frombuffer(b"".join(bytes(s) for s in seeds), dtype=np.uint8).reshape(-1, 32).copy()
    a = np.ascontiguousarray(seeds, dtype=np.uint8)
    if a.size % 32:
        raise RuntimeError("seeds must be K x 32 bytes")
    return a.reshape(-1, 32)


def _signs_array(signs, K: int) -> np.ndarray:
    s = np.ascontiguousarray(signs, dtype=np.int8).reshape(-1)
    if s.shape[0] != K:
        raise RuntimeError(f"{s.shape[0]} signs for {K} seeds")
    return s


def _need(cond: bool, msg: str):
    if not cond:
        raise RuntimeError(msg)


def _dev_bytes(t, name: str, cols: int, rows: int, dtype_bytes: int = 1):
    """A contiguous CUDA tensor of >= rows x cols elements of dtype_bytes each (the kernels index it flat)."""
    _need(t is not None and t.is_cuda and t.is_contiguous() and t.element_size() == dtype_bytes,
          f"{name} must be a contiguous CUDA tensor of {dtype_bytes}-byte elements")
    _need(t.numel() >= rows * cols and (cols == 1 or t.shape[-1] == cols),
          f"{name} must hold >= {rows} x {cols} elements, got {tuple(t.shape)}")


def _dev_rows(rows, L: int) -> int:
    """Row pitch (elements) of an (N, >= L) 32-bit CUDA tensor whose rows may be a strided view."""
    _need(rows.is_cuda and rows.dim() == 2 and rows.element_size() == 4, "rows must be a 2-D 32-bit CUDA tensor")
    _need(rows.shape[1] <= 1 or rows.stride(1) == 1, "rows must be contiguous along a row")
    pitch = rows.stride(0) if rows.shape[0] > 1 else rows.shape[1]
    _need(rows.shape[1] >= L and pitch >= rows.shape[1], f"rows must be (N, >= {L}), got {tuple(rows.shape)}")
    return pitch


class MaskEngine:
    """One GPU's mask-and-aggregate engine (a flm_ctx)."""

    def __init__(self, device: int = 0, _ctx=None):
        self.lib = _lib.load()
        self.device = device
        self._owned = _ctx is None
        if _ctx is not None:                 # a context owned by a DeviceGroup
            self.ctx = ctypes.c_void_p(_ctx)
            return
        ctx = ctypes.c_void_p()
        rc = self.lib.flm_init(ctypes.byref(ctx), device)
        if rc != 0:
            raise RuntimeError(f"flm_init(device={device}) failed: {self.lib.flm_last_error(None).decode()}")
        self.ctx = ctx

    # ------------------------------------------------------------ plumbing
    def close(self):
        if not getattr(self, "_owned", True):
            self.ctx = None
            return
        if getattr(self, "ctx", None) is not None and self.ctx.value:
            for st in self.__dict__.pop("_cu_streams", {}).values():
                st.synchronize()
                self.lib.flm_stream_destroy(self.ctx, ctypes.c_void_p(st.cuda_stream))
            self.lib.flm_free(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.flm_last_error(self.ctx).decode()} (code {rc})")

    def set_tuning(self, key: str, value: int):
        """A/B knobs (flm_set_tuning, include/flamingo_hip.h): variant, subtiles, pairing, ..."""
        self._check(self.lib.flm_set_tuning(self.ctx, key.encode(), int(value)), f"flm_set_tuning({key})")

    def get_tuning(self, key: str) -> int:
        """The context's current value of `key` (flm_get_tuning): also what another wrapper of the
        same flm_ctx (DeviceGroup engines, a direct flm_set_tuning call) set."""
        v = ctypes.c_int()
        self._check(self.lib.flm_get_tuning(self.ctx, key.encode(), ctypes.byref(v)), f"flm_get_tuning({key})")
        return v.value

    def last_plan(self) -> dict:
        v = [ctypes.c_int() for _ in range(4)]
        self.lib.flm_last_plan(self.ctx, *[ctypes.byref(x) for x in v])
        return {"items": v[0].value, "tile_slots": v[1].value, "atomics": v[2].value, "variant": v[3].value}

    def cu_count(self) -> int:
        n = ctypes.c_int()
        self._check(self.lib.flm_cu_count(self.ctx, ctypes.byref(n)), "flm_cu_count")
        return n.value

    def cu_stream(self, cus):
        """A torch ExternalStream whose kernels run only on the logical CUs in `cus`
        (flm_stream_create_cu_mask).  Cached per CU set and owned by the engine:
        destroyed by close() after a device synchronize.  Never record_stream() a
        tensor on it (the caching allocator would touch the stream after close)."""
        import torch
        cus = tuple(sorted(set(int(c) for c in cus)))
        if not cus:
            raise ValueError("cu_stream: empty CU set")
        cache = self.__dict__.setdefault("_cu_streams", {})
        if cus in cache:
            return cache[cus]
        words = np.zeros((max(cus) // 32) + 1, np.uint32)
        for c in cus:
            words[c // 32] |= np.uint32(1 << (c % 32))
        h = ctypes.c_void_p()
        self._check(self.lib.flm_stream_create_cu_mask(self.ctx, words.ctypes.data_as(ctypes.c_void_p), len(words),
                                                        ctypes.byref(h)), "flm_stream_create_cu_mask")
        cache[cus] = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", self.device))
        return cache[cus]

    # ----------------------------------------------- RCCL (one process per GPU)
    def comm_init(self, n_ranks: int, rank: int, unique_id: bytes):
        """Attach an RCCL communicator (flm_comm_init_rank; collective over all ranks)."""
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
        self._check(self.lib.flm_comm_init_rank(self.ctx, int(n_ranks), int(rank), uid), "flm_comm_init_rank")

    def comm_destroy(self):
        """Synchronise the device, then finalize + destroy the attached RCCL communicator
        (flm_comm_destroy; a no-op without one).  distributed.shutdown calls this on every rank
        before torch.distributed's process group is destroyed."""
        if getattr(self, "ctx", None) is not None and self.ctx.value:
            self._check(self.lib.flm_comm_destroy(self.ctx), "flm_comm_destroy")

    def comm_size(self):
        """(n_ranks, rank) of the attached communicator, (1, 0) without one."""
        n, r = ctypes.c_int(), ctypes.c_int()
        self.lib.flm_comm_size(self.ctx, ctypes.byref(n), ctypes.byref(r))
        return n.value, r.value

    def has_comm(self) -> bool:
        """True when an RCCL communicator is attached (flm_comm_size returns 0; 1 = none)."""
        n, r = ctypes.c_int(), ctypes.c_int()
        return self.lib.flm_comm_size(self.ctx, ctypes.byref(n), ctypes.byref(r)) == 0

    def reduce_scatter_dev(self, send, recv, recv_words: int | None = None, stream=None):
        """recv[:recv_words] = this rank's slice of sum_ranks(send) as uint32 (ncclUint32, ncclSum)."""
        n = int(recv.numel() if recv_words is None else recv_words)
        if send.numel() < n * self.comm_size()[0] or recv.numel() < n or send.element_size() != 4:
            raise RuntimeError("reduce_scatter_dev: send must hold n_ranks * recv_words 32-bit words")
        self._check(self.lib.flm_reduce_scatter_dev(self.ctx, send.data_ptr(), recv.data_ptr(), n,
                                                    self._stream_handle(stream)), "flm_reduce_scatter_dev")
        return recv

    def all_gather_dev(self, send, recv, stream=None):
        """recv = concat over ranks of send's bytes (ncclAllGather, ncclUint8)."""
        nb = send.numel() * send.element_size()
        if recv.numel() * recv.element_size() < nb * self.comm_size()[0]:
            raise RuntimeError("all_gather_dev: recv too small")
        self._check(self.lib.flm_all_gather_dev(self.ctx, send.data_ptr(), recv.data_ptr(), nb,
                                                self._stream_handle(stream)), "flm_all_gather_dev")
        return recv

    # -------------------------------------------------------- host arrays
    def aggregate_unmask(self, vectors, seeds, signs, L: int | None = None) -> np.ndarray:
        """sum(vectors) + sum_k signs[k]*PRG(seeds[k]) mod 2^32 (host in, host out).

        vectors: a list of uint32 arrays (the VECTOR bodies) or an (N, L) array."""
        if isinstance(vectors, np.ndarray) and vectors.ndim == 2:
            rows = [np.ascontiguousarray(vectors[i], dtype=np.uint32) for i in range(vectors.shape[0])]
        else:
            rows = [np.ascontiguousarray(v, dtype=np.uint32) for v in vectors]
        if L is None:
            if not rows:
                raise RuntimeError("L is required when there are no vectors")
            L = rows[0].shape[0]
        for v in rows:
            if v.shape[0] != L:
                raise RuntimeError("Client sends vector of incorrect length.")  # SA_ServiceAgent.py:348-349
        seeds = _seeds_array(seeds)
        signs = _signs_array(signs, seeds.shape[0])
        out = np.empty(L, dtype=np.uint32)
        ptrs = (_lib._u32p * max(1, len(rows)))(*[p_u32(v) for v in rows])
        rc = self.lib.flm_aggregate_unmask(self.ctx, ptrs, len(rows), p_u8(seeds), p_i8(signs), seeds.shape[0],
                                           L, p_u32(out))
        self._check(rc, "flm_aggregate_unmask")
        return out

    def client_mask(self, seg, seeds, signs, L: int, x: np.ndarray | None = None) -> np.ndarray:
        """y_i = x_i (or ones) + sum_{k in seg i} signs[k]*PRG(seeds[k]); returns (N, L) uint32."""
        seg = np.ascontiguousarray(seg, dtype=np.int64)
        N = seg.shape[0] - 1
        seeds = _seeds_array(seeds)
        signs = _signs_array(signs, seeds.shape[0])
        if seg[-1] != seeds.shape[0]:
            raise RuntimeError("seg[-1] must equal the number of seeds")
        out = np.empty((N, L), dtype=np.uint32)
        xp = None
        if x is not None:
            x = np.ascontiguousarray(x, dtype=np.uint32)
            if x.shape != (N, L):
                raise RuntimeError("x must be (N, L)")
            xp = p_u32(x)
        rc = self.lib.flm_client_mask(self.ctx, xp, N, p_i64(seg), p_u8(seeds), p_i8(signs), L, p_u32(out))
        self._check(rc, "flm_client_mask")
        return out

    def prg_expand(self, seeds, L: int, slot0: int = 0) -> np.ndarray:
        """PRG(seed_k)[slot0:slot0+L] for every seed; (K, L) uint32."""
        seeds = _seeds_array(seeds)
        out = np.empty((seeds.shape[0], L), dtype=np.uint32)
        rc = self.lib.flm_prg_expand(self.ctx, p_u8(seeds), seeds.shape[0], L, slot0, p_u32(out))
        self._check(rc, "flm_prg_expand")
        return out

    def prg(self, seed: bytes, L: int, slot0: int = 0) -> np.ndarray:
        return self.prg_expand([seed], L, slot0)[0]

    def mask_accumulate(self, seeds, signs, acc: np.ndarray, slot0: int = 0) -> np.ndarray:
        """acc += sum_k signs[k]*PRG(seeds[k])[slot0:] in place; returns acc."""
        if acc.dtype != np.uint32 or not acc.flags.c_contiguous:
            raise RuntimeError("acc must be a C-contiguous uint32 array")
        seeds = _seeds_array(seeds)
        signs = _signs_array(signs, seeds.shape[0])
        rc = self.lib.flm_mask_accumulate(self.ctx, p_u8(seeds), p_i8(signs), seeds.shape[0], p_u32(acc),
                                          acc.shape[0], slot0)
        self._check(rc, "flm_mask_accumulate")
        return acc

    def chacha20_encrypt(self, key: bytes, data: bytes, nonce: bytes = NONCE, counter: int = 0) -> bytes:
        """ChaCha20.new(key=key, nonce=nonce).encrypt(data) (DJB layout), on the GPU."""
        if len(key) != 32 or len(nonce) != 8:
            raise RuntimeError("key must be 32 bytes and nonce 8 bytes")
        n = len(data)
        if n == 0:
            return b""
        src = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        dst = np.empty(n, dtype=np.uint8)
        k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
        nn = np.frombuffer(bytes(nonce), dtype=np.uint8).copy()
        rc = self.lib.flm_chacha20_xor(self.ctx, p_u8(k), p_u8(nn), counter, p_u8(src), p_u8(dst), n)
        self._check(rc, "flm_chacha20_xor")
        return dst.tobytes()

    # ------------------------------------------------------ device tensors
    @staticmethod
    def _stream_handle(stream) -> int:
        """hipStream_t as an int (the c_void_p argtypes take ints as they are)."""
        if stream is None:
            import torch
            return torch.cuda.current_stream().cuda_stream
        if isinstance(stream, int):
            return stream
        return stream.cuda_stream

    def aggregate_unmask_dev(self, rows, seeds, signs, out, L: int | None = None, mask_lo: int = 0,
                             mask_hi: int | None = None, prg_slot0: int = 0, stream=None):
        """Enqueue the device-resident round on `stream` (default: torch's current stream).

        rows: (N, pitch) int32/uint32 CUDA tensor (pitch % 4 == 0, pitch >= L);
        seeds: (K, 32) uint8 CUDA tensor; signs: (K,) int8 CUDA tensor;
        out: CUDA tensor with >= L int32/uint32 elements."""
        # lean checks: this call is the whole host cost of a small round (c2), and every torch
        # attribute read costs ~0.3 us; the other *_dev wrappers check fully (_dev_bytes, _dev_rows)
        N = rows.shape[0] if rows is not None else 0
        width = rows.shape[1] if N else 0
        pitch = rows.stride(0) if N > 1 else width          # a strided row view keeps its true pitch
        if L is None:
            L = width
        if mask_hi is None:
            mask_hi = L
        K = seeds.shape[0] if seeds is not None else 0
        if K and (seeds.shape[-1] != 32 or signs.shape[0] < K):
            raise RuntimeError(f"seeds must be (K, 32) with >= K signs, got {tuple(seeds.shape)}, {tuple(signs.shape)}")
        if (N and width < L) or out.numel() < L:
            raise RuntimeError(f"rows must be (N, >= {L}) and out hold >= {L} elements")
        # plain ints for the c_void_p arguments: this call is the whole host cost of a small
        # round (c2: ~6.5 us of GPU time), so no per-call ctypes wrapper objects
        rc = self.lib.flm_aggregate_unmask_dev(
            self.ctx, rows.data_ptr() if N else 0, pitch, N, seeds.data_ptr() if K else 0,
            signs.data_ptr() if K else 0, K, L, mask_lo, mask_hi, prg_slot0, out.data_ptr(),
            self._stream_handle(stream))
        if rc:
            self._check(rc, "flm_aggregate_unmask_dev")
        return out

    def seed_table_dev(self, seeds, signs, stream=None):
        """Build the device seed schedule (first of the round's two launches)."""
        K = seeds.shape[0] if seeds is not None else 0
        rc = self.lib.flm_seed_table_dev(self.ctx, ctypes.c_void_p(seeds.data_ptr() if K else 0),
                                         ctypes.c_void_p(signs.data_ptr() if K else 0), K,
                                         self._stream_handle(stream))
        self._check(rc, "flm_seed_table_dev")

    def aggregate_dev(self, rows, K: int, out, L: int | None = None, mask_lo: int = 0, mask_hi: int | None = None,
                      prg_slot0: int = 0, stream=None):
        """Row-sum + unmask kernel against the current seed table (second launch)."""
        N = rows.shape[0] if rows is not None else 0
        if L is None:
            L = rows.shape[1] if N else 0
        pitch = _dev_rows(rows, L) if N else 0
        if mask_hi is None:
            mask_hi = L
        _dev_bytes(out, "out", 1, L, 4)
        rc = self.lib.flm_aggregate_dev(self.ctx, ctypes.c_void_p(rows.data_ptr() if N else 0), pitch, N, K, L,
                                        mask_lo, mask_hi, prg_slot0, ctypes.c_void_p(out.data_ptr()),
                                        self._stream_handle(stream))
        self._check(rc, "flm_aggregate_dev")
        return out

    def client_mask_dev(self, seg, seeds_dev, signs, out, L: int, x=None, stream=None):
        """Device client masking: seg/signs host arrays, seeds_dev/x/out CUDA tensors (rows at out.shape[1])."""
        seg = np.ascontiguousarray(seg, dtype=np.int64)
        N = seg.shape[0] - 1
        signs = np.ascontiguousarray(signs, dtype=np.int8)
        K = int(seg[-1]) if N >= 0 else 0
        # the C side reads signs[0..seg[N]) from this host array and indexes the device seed
        # table by seg: check both here, where the shapes are known
        if N < 0 or seg[0] != 0 or np.any(np.diff(seg) < 0):
            raise RuntimeError("seg must be non-decreasing from 0")
        if signs.ndim != 1 or signs.shape[0] != K:
            raise RuntimeError(f"{signs.shape[0] if signs.ndim else 0} signs for seg[-1] = {K} seeds")
        if K and (seeds_dev.dim() != 2 or seeds_dev.shape[1] != 32 or seeds_dev.element_size() != 1
                  or seeds_dev.shape[0] < K):
            raise RuntimeError(f"seeds_dev must be a (>= {K}, 32) uint8 tensor, got {tuple(seeds_dev.shape)}")
        if out.dim() != 2 or out.shape[0] < N or out.element_size() != 4 or out.shape[1] < L:
            raise RuntimeError(f"out must be (>= {N}, >= {L}) 32-bit, got {tuple(out.shape)}")
        if x is not None and (tuple(x.shape) != tuple(out.shape) or x.element_size() != 4):
            raise RuntimeError("x must have out's shape and a 32-bit dtype")
        pitch = out.shape[1]
        rc = self.lib.flm_client_mask_dev(self.ctx, ctypes.c_void_p(x.data_ptr() if x is not None else 0), pitch, N,
                                          p_i64(seg), ctypes.c_void_p(seeds_dev.data_ptr()), p_i8(signs), L,
                                          ctypes.c_void_p(out.data_ptr()), self._stream_handle(stream))
        self._check(rc, "flm_client_mask_dev")
        return out

    def prg_expand_dev(self, seeds_dev, out, L: int, slot0: int = 0, stream=None):
        K = seeds_dev.shape[0]
        rc = self.lib.flm_prg_expand_dev(self.ctx, ctypes.c_void_p(seeds_dev.data_ptr()), K, L, slot0,
                                         ctypes.c_void_p(out.data_ptr()), out.shape[1], self._stream_handle(stream))
        self._check(rc, "flm_prg_expand_dev")
        return out

    # ------------------------------------------------------------ P-256
    def ec_mul_wire(self, points_w: np.ndarray, scalars_w: np.ndarray):
        """Batched k_i * P_i on wire arrays: points (n, 64) and scalars (n, 32) uint8 big endian.
        Returns (out (n, 64) uint8, flags (n,) uint32; bit 2 = infinity, returned as zeros)."""
        pw = np.ascontiguousarray(points_w, np.uint8).reshape(-1, 64)
        sw = np.ascontiguousarray(scalars_w, np.uint8).reshape(-1, 32)
        n = pw.shape[0]
        if sw.shape[0] != n:
            raise RuntimeError(f"{sw.shape[0]} scalars for {n} points")
        out = np.zeros((n, 64), np.uint8)
        fl = np.zeros(n, np.uint32)
        if n:
            self._check(self.lib.flm_ec_mul(self.ctx, p_u8(pw), p_u8(sw), n, p_u8(out), p_u32(fl)), "flm_ec_mul")
        return out, fl

    def hash_to_curve_wire(self, msgs):
        """ecchash.hash_str_to_curve(msg, 2, n, 1, 48, XMD SHA-256) of each message (str or bytes,
        <= 64 bytes) on the GPU (flm_hash_to_curve).  Returns (out (n, 64) uint8 wire x||y,
        flags (n,) uint32; bit 2 = infinity)."""
        raw = [m.encode() if isinstance(m, str) else bytes(m) for m in msgs]
        n = len(raw)
        buf = np.zeros((max(n, 1), 64), np.uint8)
        lens = np.zeros(max(n, 1), np.uint32)
        for i, m in enumerate(raw):
            if len(m) > 64:
                raise RuntimeError(f"message {i} is {len(m)} bytes (at most 64)")
            buf[i, :len(m)] = np.frombuffer(m, np.uint8)
            lens[i] = len(m)
        out = np.zeros((n, 64), np.uint8)
        fl = np.zeros(n, np.uint32)
        if n:
            self._check(self.lib.flm_hash_to_curve(self.ctx, p_u8(buf), p_u32(lens), n, p_u8(out), p_u32(fl)),
                        "flm_hash_to_curve")
        return out, fl

    def hash_to_curve_decimal(self, v0: int = 0, n: int = 1 << 16):
        """hash_str_to_curve(str(v)) for v in [v0, v0 + n) in one launch (flm_hash_to_curve_decimal):
        with the defaults, every h_ijt a client can hash (SA_ClientAgent.py:280).  (out, flags) as
        hash_to_curve_wire."""
        out = np.zeros((n, 64), np.uint8)
        fl = np.zeros(n, np.uint32)
        if n:
            self._check(self.lib.flm_hash_to_curve_decimal(self.ctx, int(v0), int(n), p_u8(out), p_u32(fl)),
                        "flm_hash_to_curve_decimal")
        return out, fl

    def hash_to_curve_decimal_dev(self, v0: int, n: int, out, flags, stream=None):
        """Device form: out (n, 64) uint8 and flags (n,) int32/uint32 CUDA tensors; enqueued on `stream`."""
        _dev_bytes(out, "out", 64, n)
        _dev_bytes(flags, "flags", 1, n, 4)
        self._check(self.lib.flm_hash_to_curve_decimal_dev(self.ctx, int(v0), int(n), out.data_ptr(), flags.data_ptr(),
                                                           self._stream_handle(stream)),
                    "flm_hash_to_curve_decimal_dev")
        return out, flags

    def ec_mul(self, points, scalars) -> list:
        """[k_i * P_i] for affine points (x, y) and integer scalars (flm_ec_mul).

        The ECDH / ElGamal / decryption-share products of SA_ClientAgent.py:256-263,
        :434-447 and :397-400, batched.  Infinity comes back as None."""
        from .crypto import points_from_wire, points_to_wire, scalars_to_wire
        if len(scalars) != len(points):
            raise RuntimeError(f"{len(scalars)} scalars for {len(points)} points")
        if not points:
            return []
        out, fl = self.ec_mul_wire(points_to_wire(points), scalars_to_wire(scalars))
        return points_from_wire(out, fl)

    def ec_combine_wire(self, c1_w, shares_w, lambdas_w, negate: bool = True):
        """flm_ec_combine on wire arrays: c1 (D, 64) or None, shares (T, D, 64), lambdas (T, 32).
        Returns (points (D, 64), seeds (D, 32), flags (D,))."""
        sh = np.ascontiguousarray(shares_w, np.uint8)
        T = sh.shape[0]
        lw = np.ascontiguousarray(lambdas_w, np.uint8).reshape(-1, 32)
        if lw.shape[0] != T:
            raise RuntimeError(f"{lw.shape[0]} coefficients for {T} share sets")
        D = c1_w.shape[0] if c1_w is not None else (sh.shape[1] if T else 0)
        if T and (sh.ndim != 3 or sh.shape[1] != D or sh.shape[2] != 64):
            raise RuntimeError("shares must be (T, D, 64)")
        pts = np.zeros((D, 64), np.uint8)
        seeds = np.zeros((D, 32), np.uint8)
        fl = np.zeros(D, np.uint32)
        if D == 0:
            return pts, seeds, fl
        cw = np.ascontiguousarray(c1_w, np.uint8) if c1_w is not None else None
        if not T:
            sh, lw = np.zeros((1, 64), np.uint8), np.zeros((1, 32), np.uint8)
        rc = self.lib.flm_ec_combine(self.ctx, p_u8(cw) if cw is not None else None, p_u8(sh), p_u8(lw), T, D,
                                     1 if negate else 0, p_u8(pts), p_u8(seeds), p_u32(fl))
        self._check(rc, "flm_ec_combine")
        return pts, seeds, fl

    def ec_combine(self, c1, shares_by_term, lambdas, negate: bool = True):
        """Threshold-ElGamal combine + seed derivation (SA_ServiceAgent.py:542-585).

        c1: D affine points (or None: base = infinity); shares_by_term: T lists of D
        points (share_{j,i} = sk_j * c0_i); lambdas: T Lagrange coefficients.
        Returns (points, seeds): point_i = c1_i - sum_j lambda_j share_{j,i}
        (+ when negate is False) and seed_i = SHA-256(x||y) as 32 bytes."""
        from .crypto import points_from_wire, points_to_wire, scalars_to_wire
        T = len(lambdas)
        D = len(c1) if c1 is not None else (len(shares_by_term[0]) if T else 0)
        if len(shares_by_term) != T or any(len(s) != D for s in shares_by_term):
            raise RuntimeError("shares must be T lists of D points")
        if D == 0:
            return [], []
        sh = np.stack([points_to_wire(s) for s in shares_by_term]) if T else np.zeros((0, D, 64), np.uint8)
        lw = scalars_to_wire(lambdas) if T else np.zeros((0, 32), np.uint8)
        pts, seeds, fl = self.ec_combine_wire(points_to_wire(c1) if c1 is not None else None, sh, lw, negate)
        return points_from_wire(pts, fl), [bytes(r) for r in seeds]

    def shamir_combine(self, shares_by_term, lambdas) -> list:
        """m_i = sum_j lambda_j y_{j,i} mod n as 32-byte big-endian seeds (SA_ServiceAgent.py:506-526).
        shares_by_term: T sequences of M integers (< 2^256); lambdas: T integers (< n)."""
        from .crypto import scalars_to_wire
        T = len(lambdas)
        if len(shares_by_term) != T:
            raise RuntimeError(f"{len(shares_by_term)} share lists for {T} coefficients")
        M = len(shares_by_term[0]) if T else 0
        if any(len(s) != M for s in shares_by_term):
            raise RuntimeError("share lists differ in length")
        if M == 0:
            return []
        sh = np.stack([scalars_to_wire(s) for s in shares_by_term])
        out = np.zeros((M, 32), np.uint8)
        rc = self.lib.flm_shamir_combine(self.ctx, p_u8(sh), p_u8(scalars_to_wire(lambdas)), T, M, p_u8(out))
        self._check(rc, "flm_shamir_combine")
        return [bytes(r) for r in out]

    def shamir_combine_dev(self, shares, lambdas, seeds_out, stream=None):
        """Device form: shares (T, M, 32), lambdas (T, 32) uint8 CUDA tensors -> seeds_out (M, 32)."""
        _need(shares.dim() == 3, "shares must be (T, M, 32)")
        T, M = shares.shape[0], shares.shape[1]
        _dev_bytes(shares, "shares", 32, T * M)
        _dev_bytes(lambdas, "lambdas", 32, T)
        _dev_bytes(seeds_out, "seeds_out", 32, M)
        rc = self.lib.flm_shamir_combine_dev(self.ctx, ctypes.c_void_p(shares.data_ptr()),
                                             ctypes.c_void_p(lambdas.data_ptr()), T, M,
                                             ctypes.c_void_p(seeds_out.data_ptr()), self._stream_handle(stream))
        self._check(rc, "flm_shamir_combine_dev")
        return seeds_out

    def ec_combine_dev(self, c1, shares, lambdas, seeds_out, flags, points_out=None, negate: bool = True,
                       stream=None):
        """Device form: c1 (D,64), shares (T,D,64), lambdas (T,32) uint8 CUDA tensors;
        seeds_out (D,32) uint8 and flags (D,) int32 CUDA tensors are written on `stream`."""
        _need(shares.dim() == 3, "shares must be (T, D, 64)")
        T, D = shares.shape[0], shares.shape[1]
        _dev_bytes(shares, "shares", 64, T * D)
        _dev_bytes(lambdas, "lambdas", 32, T)
        if c1 is not None:
            _dev_bytes(c1, "c1", 64, D)
        if seeds_out is not None:
            _dev_bytes(seeds_out, "seeds_out", 32, D)
        if points_out is not None:
            _dev_bytes(points_out, "points_out", 64, D)
        _dev_bytes(flags, "flags", 1, D, 4)
        vp = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
        rc = self.lib.flm_ec_combine_dev(self.ctx, vp(c1), vp(shares), vp(lambdas), T, D, 1 if negate else 0,
                                         vp(points_out), vp(seeds_out), vp(flags), self._stream_handle(stream))
        self._check(rc, "flm_ec_combine_dev")
        return seeds_out

    def pair_units_dev(self, seeds, signs, dst, L: int, ws, groups: int, p0=None, p1=None, final: bool = False,
                       stream=None):
        """Pair masks as a shared work queue (flm_pair_units_dev): seeds (K,32) uint8, signs (K,) int8,
        dst (>= L) int32, ws (>= 2) int32 CUDA tensors.  final=False adds the units claimed before
        ws[1] is set into dst; final=True writes dst = p0 + p1 plus the units left."""
        K = seeds.shape[0] if seeds is not None else 0
        if K:
            _dev_bytes(seeds, "seeds", 32, K)
            _dev_bytes(signs, "signs", 1, K)
        _dev_bytes(dst, "dst", 1, L, 4)
        _dev_bytes(ws, "ws", 1, 2, 4)
        for name, t in (("p0", p0), ("p1", p1)):
            if t is not None:
                _dev_bytes(t, name, 1, L, 4)
        vp = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
        rc = self.lib.flm_pair_units_dev(self.ctx, vp(seeds), vp(signs), K, vp(p0), vp(p1), vp(dst), L, vp(ws),
                                         1 if final else 0, int(groups), self._stream_handle(stream))
        self._check(rc, "flm_pair_units_dev")
        return dst

    def flag_set_dev(self, ws, stream=None):
        """ws[1] = 1 once the work enqueued before it on `stream` is done (flm_flag_set_dev)."""
        self._check(self.lib.flm_flag_set_dev(self.ctx, ctypes.c_void_p(ws.data_ptr()), self._stream_handle(stream)),
                    "flm_flag_set_dev")

    def check_signs(self) -> int:
        bad = ctypes.c_int()
        self._check(self.lib.flm_check_signs(self.ctx, ctypes.byref(bad)), "flm_check_signs")
        return bad.value


class PinnedArena:
    """Page-locked host memory (hipHostMalloc) viewed as numpy arrays.

    Client vectors allocated here reach the GPU by DMA at the full PCIe rate
    (the reference keeps them as pageable numpy arrays, SA_ServiceAgent.py:210)."""

    def __init__(self, nbytes: int):
        self.lib = _lib.load()
        self.ptr = self.lib.flm_host_alloc(nbytes)
        if not self.ptr:
            raise RuntimeError(f"flm_host_alloc({nbytes}) failed")
        self.nbytes = nbytes
        self.off = 0

    def array(self, shape, dtype=np.uint32) -> np.ndarray:
        dt = np.dtype(dtype)
        n = int(np.prod(shape)) * dt.itemsize
        off = (self.off + 255) // 256 * 256
        if off + n > self.nbytes:
            raise RuntimeError("pinned arena exhausted")
        self.off = off + n
        buf = (ctypes.c_uint8 * n).from_address(self.ptr + off)
        return np.frombuffer(buf, dtype=dt).reshape(shape)

    def free(self):
        if self.ptr:
            self.lib.flm_host_free(self.ptr)
            self.ptr = None


# ------------------------------------------------------------------ multi-GPU
def rccl_available():
    """(True, "") when RCCL loads and resolves (flm_rccl_available; local, no GPU work), else (False, why)."""
    lib = _lib.load()
    if lib.flm_rccl_available():
        return True, ""
    return False, lib.flm_last_error(None).decode()


def comm_unique_id() -> bytes:
    """A fresh 128-byte RCCL unique id (flm_comm_unique_id), for rank 0 to broadcast."""
    lib = _lib.load()
    buf = (ctypes.c_uint8 * 128)()
    rc = lib.flm_comm_unique_id(buf)
    if rc != 0:
        raise RuntimeError(f"flm_comm_unique_id: {lib.flm_last_error(None).decode()}")
    return bytes(buf)


def shard_bounds(L: int, n_ranks: int, rank: int):
    """(lo, hi, S): rank's output slots [lo, hi) and the shard length S (flm_shard_bounds)."""
    lib = _lib.load()
    lo, hi, S = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    if lib.flm_shard_bounds(int(L), int(n_ranks), int(rank), ctypes.byref(lo), ctypes.byref(hi), ctypes.byref(S)):
        raise RuntimeError("flm_shard_bounds: bad arguments")
    return lo.value, hi.value, S.value


def client_bounds(N: int, n_ranks: int, rank: int):
    """[c0, c1): the clients rank ingests (flm_client_bounds)."""
    lib = _lib.load()
    c0, c1 = ctypes.c_int(), ctypes.c_int()
    if lib.flm_client_bounds(int(N), int(n_ranks), int(rank), ctypes.byref(c0), ctypes.byref(c1)):
        raise RuntimeError("flm_client_bounds: bad arguments")
    return c0.value, c1.value


class DeviceGroup:
    """All GPUs of the node from ONE process (flm_group): the drop-in server's multi-GPU form.

    The reference server is a single-threaded DES process (Kernel.py:190-271); a group gives
    its report/reconstruction steps every device: client-sharded upload and row sum,
    slot-sharded unmask, one RCCL reduce-scatter (ncclUint32), shards back to the host.
    devices: distinct ids (RCCL clique) or one id repeated (loopback ranks on one GPU).
    force_rccl: give a one-device group an RCCL clique too (FLM_GROUP_RCCL), so its rounds take
    the multi-GPU path -- partial buffer, grouped ncclReduceScatter, shard -- on a one-GPU box."""

    def __init__(self, devices, force_rccl: bool = False):
        self.lib = _lib.load()
        if isinstance(devices, int):
            devices = list(range(devices))
        devices = [int(d) for d in devices]
        arr = (ctypes.c_int * len(devices))(*devices)
        g = ctypes.c_void_p()
        rc = self.lib.flm_group_init_flags(ctypes.byref(g), len(devices), arr, 1 if force_rccl else 0)
        if rc != 0:
            raise RuntimeError(f"flm_group_init({devices}): {self.lib.flm_group_last_error(None).decode()}")
        self.g = g
        self.devices = devices
        self.n = len(devices)
        self.loopback = bool(self.lib.flm_group_is_loopback(g))
        self.rccl = bool(self.lib.flm_group_has_rccl(g))
        self.force_rccl = bool(force_rccl)  # as requested (a group of distinct devices has a clique anyway)
        self._stores = 0                    # live VectorStores on this group (close() refuses while > 0)
        self.retired = False                # replaced while a store still used it: its last store closes it
        self.engines = [MaskEngine(d, _ctx=self.lib.flm_group_ctx(g, r)) for r, d in enumerate(devices)]

    def close(self):
        """Free the group.  Refused while a VectorStore created on it is still open: the store holds
        the group's contexts and streams (close the stores first)."""
        if getattr(self, "g", None) is not None and self.g.value:
            if self._stores:
                raise RuntimeError(f"DeviceGroup.close: {self._stores} VectorStore(s) still use this group")
            for e in self.engines:
                e.close()
            self.lib.flm_group_free(self.g)
            self.g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.flm_group_last_error(self.g).decode()} (code {rc})")

    def sync(self):
        self._check(self.lib.flm_group_sync(self.g), "flm_group_sync")

    def aggregate_unmask(self, vectors, seeds, signs, L: int | None = None) -> np.ndarray:
        """MaskEngine.aggregate_unmask over every device of the group (host rows in, host out)."""
        if isinstance(vectors, np.ndarray) and vectors.ndim == 2:
            rows = [np.ascontiguousarray(vectors[i], dtype=np.uint32) for i in range(vectors.shape[0])]
        else:
            rows = [np.ascontiguousarray(v, dtype=np.uint32) for v in vectors]
        if L is None:
            if not rows:
                raise RuntimeError("L is required when there are no vectors")
            L = rows[0].shape[0]
        for v in rows:
            if v.shape[0] != L:
                raise RuntimeError("Client sends vector of incorrect length.")  # SA_ServiceAgent.py:348-349
        seeds = _seeds_array(seeds)
        signs = _signs_array(signs, seeds.shape[0])
        out = np.empty(L, dtype=np.uint32)
        ptrs = (_lib._u32p * max(1, len(rows)))(*[p_u32(v) for v in rows])
        self._check(self.lib.flm_group_aggregate_unmask(self.g, ptrs, len(rows), p_u8(seeds), p_i8(signs),
                                                        seeds.shape[0], L, p_u32(out)),
                    "flm_group_aggregate_unmask")
        return out

    def rank_stream(self, r: int):
        """Rank r's context stream (flm_ctx_stream) as a torch ExternalStream: the group's rounds run there."""
        import torch
        cache = self.__dict__.setdefault("_rank_streams", {})
        if r not in cache:
            h = self.lib.flm_ctx_stream(self.lib.flm_group_ctx(self.g, r))
            cache[r] = torch.cuda.ExternalStream(h, device=torch.device("cuda", self.devices[r]))
        return cache[r]

    def wait(self):
        """Make torch's current stream on every rank's device wait for that rank's round
        (no host synchronisation): the shards can then be read in stream order."""
        import torch
        for r, d in enumerate(self.devices):
            torch.cuda.current_stream(torch.device("cuda", d)).wait_stream(self.rank_stream(r))

    def aggregate_unmask_dev(self, rows, seeds, signs, shards, L: int, after_current: bool = True):
        """rows/seeds/signs/shards: per-rank CUDA tensors on the ranks' devices (rows (N_r, pitch) with one
        common pitch; shards >= S words).  Enqueued on the ranks' context streams and returns.
        after_current: each rank's stream first waits for torch's current stream on its device, where
        the inputs were produced (False: the caller has ordered them itself).  Read the shards after
        sync() (host) or wait() (torch's current streams)."""
        n = self.n
        _need(len(rows) == n and len(shards) == n and len(seeds) == n and len(signs) == n,
              f"rows, seeds, signs and shards need one entry per rank ({n})")
        pitches = {_dev_rows(r, L) for r in rows if r is not None and r.shape[0]}
        _need(len(pitches) <= 1, f"every rank's rows need the same pitch, got {sorted(pitches)}")
        pitch = pitches.pop() if pitches else 0
        K = seeds[0].shape[0] if seeds and seeds[0] is not None else 0
        S = shard_bounds(L, n, 0)[2]
        for r in range(n):
            if K:
                _dev_bytes(seeds[r], f"seeds[{r}]", 32, K)
                _need(seeds[r].shape[0] == K, "every rank needs the same K seeds")
                _dev_bytes(signs[r], f"signs[{r}]", 1, K)
            _dev_bytes(shards[r], f"shards[{r}]", 1, S, 4)
        vp = ctypes.c_void_p
        d_rows = (vp * n)(*[r.data_ptr() if r is not None and r.shape[0] else 0 for r in rows])
        n_rows = (ctypes.c_int * n)(*[int(r.shape[0]) if r is not None else 0 for r in rows])
        d_seeds = (vp * n)(*[s.data_ptr() if K else 0 for s in seeds])
        d_signs = (vp * n)(*[s.data_ptr() if K else 0 for s in signs])
        d_shards = (vp * n)(*[s.data_ptr() for s in shards])
        if after_current:
            import torch
            for r, d in enumerate(self.devices):
                self.rank_stream(r).wait_stream(torch.cuda.current_stream(torch.device("cuda", d)))
        self._check(self.lib.flm_group_aggregate_unmask_dev(self.g, d_rows, pitch, n_rows, d_seeds, d_signs, K, L,
                                                            d_shards), "flm_group_aggregate_unmask_dev")
        return shards
