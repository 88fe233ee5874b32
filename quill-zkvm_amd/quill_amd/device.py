"""Device context, SRS and device-resident Fr vectors (qg_ctx / qg_srs / qg_buf)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import check, lib
from .field import fr_array, fr_c, fr_list, g1_from_abi, g1_to_abi, u64p

_NO_POOL = os.environ.get("QG_NO_POOL") == "1"  # A/B runs: every buffer freed on close


class Device:
    """One HIP device (qg_ctx_create).  Context for every GPU call."""

    def __init__(self, device: int = 0):
        self.h = C.c_void_p()
        check(lib().qg_ctx_create(device, C.byref(self.h)))
        self.device = device
        self.rank, self.world = 0, 1
        # freed pooled buffers by length (DeviceVec(..., pooled=True)): a prover's
        # per-proof temporaries are reused instead of hipFree'd, which waits for
        # the device to drain and then costs ~0.2 ms of host time each
        self._pool = {}

    def close(self):
        if self.h:
            for hs in self._pool.values():
                for h in hs:
                    lib().qg_buf_destroy(h)
            self._pool = {}
            lib().qg_ctx_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def attach_comm(self, rank: int, world: int, unique_id: bytes = None):
        """RCCL communicator (qg_ctx_attach_comm); world 1 detaches unless
        QG_FORCE_RCCL=1 (then a one-rank RCCL communicator, unique_id optional)"""
        buf = None if unique_id is None else (C.c_uint8 * 128).from_buffer_copy(unique_id)
        check(lib().qg_ctx_attach_comm(self.h, rank, world, buf), self.h)
        self.rank, self.world = rank, world

    def comm_info(self) -> dict:
        """{"kind": "none" | "loopback" | "rccl", "rank", "world", "sharded"}"""
        k, r, w, s = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        check(lib().qg_ctx_comm_info(self.h, C.byref(k), C.byref(r), C.byref(w), C.byref(s)),
              self.h)
        return {"kind": ("none", "loopback", "rccl")[k.value], "rank": r.value,
                "world": w.value, "sharded": bool(s.value)}

    def alltoall_bytes(self, chunks: list) -> list:
        """personalised exchange (qg_comm_alltoall_host): chunks[d] goes to rank d
        (equal lengths); returns the chunk received from every rank, in rank order"""
        assert len(chunks) == self.world and len({len(c) for c in chunks}) == 1
        n = len(chunks[0])
        src = C.create_string_buffer(b"".join(chunks), n * self.world)
        dst = C.create_string_buffer(n * self.world)
        check(lib().qg_comm_alltoall_host(self.h, src, n, dst), self.h)
        raw = dst.raw
        return [raw[i * n:(i + 1) * n] for i in range(self.world)]

    def trace_marker(self, tag: int):
        """an empty kernel of `tag` work-groups on the context stream: cuts a
        rocprofv3 kernel trace into phases (profiles/kstats.py --legs)"""
        check(lib().qg_trace_marker(self.h, tag), self.h)

    def counter(self, name: str) -> int:
        """diagnostic counter of the context (qg_ctx_counter)"""
        v = C.c_uint64()
        check(lib().qg_ctx_counter(self.h, name.encode(), C.byref(v)), self.h)
        return v.value

    def attach_loopback(self, group, rank: int, world: int = None):
        check(lib().qg_ctx_attach_loopback(self.h, group, rank), self.h)
        self.rank = rank
        self.world = world if world is not None else self._loopback_worlds.get(
            group.value if hasattr(group, "value") else group, 1)

    _loopback_worlds = {}

    def allgather_bytes(self, data: bytes) -> list:
        """every rank's `data` (equal lengths), in rank order (qg_comm_allgather_host)"""
        n = len(data)
        if n == 0:
            return [bytes(data)] * self.world
        src = C.create_string_buffer(bytes(data), n)
        dst = C.create_string_buffer(n * self.world)
        check(lib().qg_comm_allgather_host(self.h, src, n, dst), self.h)
        raw = dst.raw
        return [raw[i * n:(i + 1) * n] for i in range(self.world)]

    @staticmethod
    def loopback_group(world: int):
        g = C.c_void_p()
        check(lib().qg_loopback_create(world, C.byref(g)))
        Device._loopback_worlds[g.value] = world
        return g

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        check(lib().qg_comm_unique_id(buf))
        return bytes(buf)

    def enable_timing(self, on=True):
        check(lib().qg_ctx_enable_timing(self.h, 1 if on else 0), self.h)

    def microbench_fq_mul(self) -> float:
        r = C.c_double()
        check(lib().qg_microbench_fq_mul(self.h, C.byref(r)), self.h)
        return r.value

    def microbench_fetch(self, rows: int, gathers: int) -> tuple:
        """(gather ms, stream ms) of the FETCH_SIZE calibration kernels"""
        g, t = C.c_double(), C.c_double()
        check(lib().qg_microbench_fetch(self.h, rows, gathers, C.byref(g), C.byref(t)), self.h)
        return g.value, t.value

    def kernel_time(self, name: str):
        ms = C.c_double()
        n = C.c_uint32()
        check(lib().qg_ctx_kernel_time(self.h, name.encode(), C.byref(ms), C.byref(n)), self.h)
        return ms.value, n.value

    def phase_split(self, names) -> dict:
        """additive device-busy ms per phase (qg_ctx_phase_split): overlapped
        intervals shared evenly, so the values sum to the busy time"""
        k = len(names)
        arr = (C.c_char_p * max(k, 1))(*[n.encode() for n in names])
        out = (C.c_double * max(k, 1))()
        check(lib().qg_ctx_phase_split(self.h, arr, k, out), self.h)
        return {n: out[i] for i, n in enumerate(names)}

    # ---- device math building blocks (mlpcs.rs / ipa.rs / eq_eval.rs) ----
    def eq_table_dev(self, point, out: "DeviceVec" = None) -> "DeviceVec":
        """fast_eq_eval_hypercube (eq_eval.rs:6-31) into a device vector"""
        n = len(point)
        pt = fr_array(point) if n else np.zeros((1, 4), dtype=np.uint64)
        out = out if out is not None else DeviceVec(self, (1 << n) // self.world, pooled=True)
        check(lib().qg_eq_table_dev(self.h, u64p(pt), n, out.h), self.h)
        return out

    def eq_table(self, point):
        n = len(point)
        pt = fr_array(point)
        out = np.zeros((1 << n, 4), dtype=np.uint64)
        check(lib().qg_eq_table(self.h, u64p(pt), n, u64p(out)), self.h)
        return fr_list(out)

    def s_polynomial(self, f, g):
        M = max(len(f), len(g))
        fa, ga = fr_array(f), fr_array(g)
        out = np.zeros((max(M - 1, 1), 4), dtype=np.uint64)
        check(lib().qg_s_polynomial(self.h, u64p(fa), len(f), u64p(ga), len(g), u64p(out)), self.h)
        return fr_list(out[:max(M - 1, 0)])

    def inner_product(self, f, g):
        fa, ga = fr_array(f), fr_array(g)
        out = (C.c_uint64 * 4)()
        check(lib().qg_inner_product(self.h, u64p(fa), len(f), u64p(ga), len(g), out), self.h)
        from .field import fr_from_mont_limbs
        return fr_from_mont_limbs(list(out))


class DeviceVec:
    """Fr vector resident in HBM (qg_buf)."""

    def __init__(self, dev: Device, n: int, pooled: bool = False):
        """pooled: the buffer comes from / returns to the device's pool of freed
        buffers of this length (contents undefined, like a fresh allocation)"""
        self.dev = dev
        self.n = n
        self.base = None  # the owning buffer when this is a view
        self.pooled = pooled and not _NO_POOL
        free = dev._pool.get(n) if self.pooled else None
        if free:
            self.h = free.pop()
        else:
            self.h = C.c_void_p()
            check(lib().qg_buf_create(dev.h, n, C.byref(self.h)), dev.h)

    def view(self, offset: int, n: int) -> "DeviceVec":
        """Entries [offset, offset+n) without a copy (qg_buf_view); keeps this
        buffer alive."""
        v = DeviceVec.__new__(DeviceVec)
        v.dev, v.n, v.base, v.pooled = self.dev, n, self, False
        v.h = C.c_void_p()
        check(lib().qg_buf_view(self.h, offset, n, C.byref(v.h)), self.dev.h)
        return v

    @classmethod
    def from_canonical(cls, dev: Device, limbs: np.ndarray, out: "DeviceVec" = None,
                       offset: int = 0):
        """(n, 4) uint64 canonical little-endian limbs (values < r) ->
        Montgomery on the device (qg_buf_upload_canonical)."""
        limbs = np.ascontiguousarray(limbs, dtype=np.uint64)
        n = limbs.shape[0]
        v = out if out is not None else cls(dev, n)
        check(lib().qg_buf_upload_canonical(v.h, offset, u64p(limbs), n), dev.h)
        return v

    @classmethod
    def from_u64(cls, dev: Device, vals, out: "DeviceVec" = None, offset: int = 0):
        """F::from(u64) of every value (qg_buf_upload_u64)."""
        arr = np.ascontiguousarray(vals, dtype=np.uint64)
        v = out if out is not None else cls(dev, arr.shape[0])
        check(lib().qg_buf_upload_u64(v.h, offset, arr.ctypes.data_as(C.POINTER(C.c_uint64)),
                                      arr.shape[0]), dev.h)
        return v

    def copy_from(self, src: "DeviceVec", dst_off: int = 0, src_off: int = 0, n: int = None):
        n = src.n - src_off if n is None else n
        check(lib().qg_buf_copy(self.h, dst_off, src.h, src_off, n), self.dev.h)
        return self

    def first_mismatch(self, other: "DeviceVec", off: int = 0, other_off: int = 0,
                       n: int = None) -> int:
        """first i with self[off+i] != other[other_off+i], or -1"""
        n = self.n - off if n is None else n
        r = C.c_int64()
        check(lib().qg_buf_first_mismatch(self.h, off, other.h, other_off, n, C.byref(r)),
              self.dev.h)
        return r.value

    @classmethod
    def from_list(cls, dev: Device, xs):
        v = cls(dev, len(xs))
        arr = fr_array(xs)
        check(lib().qg_buf_upload(v.h, u64p(arr), len(xs)), dev.h)
        return v

    def __len__(self):
        return self.n

    def fill_random(self, seed: int):
        check(lib().qg_buf_fill_random(self.h, seed), self.dev.h)
        return self

    def to_numpy(self, n=None):
        """raw Montgomery limbs, shape (n, 4) uint64"""
        n = self.n if n is None else n
        out = np.zeros((max(n, 1), 4), dtype=np.uint64)
        check(lib().qg_buf_download(self.h, u64p(out), n), self.dev.h)
        return out[:n]

    def to_list(self, n=None):
        return fr_list(self.to_numpy(n))

    def close(self):
        if self.h:
            if getattr(self, "pooled", False) and self.dev.h:
                self.dev._pool.setdefault(self.n, []).append(self.h)
            else:
                lib().qg_buf_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Srs:
    """Device-resident G1 bases (KZG::g1_points) + MSM window tables."""

    def __init__(self, dev: Device, handle):
        self.dev = dev
        self.h = handle

    @classmethod
    def generate(cls, dev: Device, tau: int, n: int, g=None, offset: int = 0):
        """bases [tau^(offset+i)] g, i < n (g = BN254 generator by default)"""
        h = C.c_void_p()
        gxy = None
        if g is not None:
            gxy, _ = g1_to_abi(g)
        check(lib().qg_srs_generate_range(dev.h, fr_c(tau), gxy, offset, n, C.byref(h)), dev.h)
        return cls(dev, h)

    @classmethod
    def upload(cls, dev: Device, points, oneshot: bool = False):
        """bases from oracle points (None = infinity).  oneshot: qg_bases_upload
        (one table, for bases that serve a single MSM) instead of the
        window-shifted tables of qg_srs_upload"""
        n = len(points)
        xy = np.zeros((n, 8), dtype=np.uint64)
        inf = np.zeros(n, dtype=np.uint8)
        for i, P in enumerate(points):
            a, f = g1_to_abi(P)
            xy[i, :] = list(a)
            inf[i] = f
        return cls.upload_raw(dev, xy, inf, oneshot)

    @classmethod
    def upload_raw(cls, dev: Device, xy: np.ndarray, inf: np.ndarray, oneshot: bool = False):
        """bases as ABI limbs: (n, 8) uint64 x||y Montgomery + (n,) uint8 flags"""
        xy = np.ascontiguousarray(xy, dtype=np.uint64)
        inf = np.ascontiguousarray(inf, dtype=np.uint8)
        h = C.c_void_p()
        fn = lib().qg_bases_upload if oneshot else lib().qg_srs_upload
        check(fn(dev.h, u64p(xy), inf.ctypes.data_as(C.POINTER(C.c_uint8)), xy.shape[0],
                 C.byref(h)), dev.h)
        return cls(dev, h)

    def __len__(self):
        return lib().qg_srs_len(self.h)

    def window_info(self):
        """(c, W): signed-digit window bits and window count"""
        c, w = C.c_int(), C.c_int()
        check(lib().qg_srs_window_info(self.h, C.byref(c), C.byref(w)), self.dev.h)
        return c.value, w.value

    def download_raw(self, offset=0, n=None):
        """affine Montgomery limbs (n, 8) uint64 + infinity flags (n,) uint8"""
        n = len(self) - offset if n is None else n
        xy = np.zeros((max(n, 1), 8), dtype=np.uint64)
        inf = np.zeros(max(n, 1), dtype=np.uint8)
        check(lib().qg_srs_download(self.h, offset, n, u64p(xy),
                                    inf.ctypes.data_as(C.POINTER(C.c_uint8))), self.dev.h)
        return xy[:n], inf[:n]

    def download(self, offset=0, n=None):
        xy, inf = self.download_raw(offset, n)
        return [g1_from_abi(xy[i], inf[i]) for i in range(len(inf))]

    def msm(self, scalars):
        arr = fr_array(scalars) if len(scalars) else np.zeros((1, 4), dtype=np.uint64)
        xy = (C.c_uint64 * 8)()
        inf = C.c_uint8()
        check(lib().qg_msm_g1(self.dev.h, self.h, u64p(arr), len(scalars), xy, C.byref(inf)),
              self.dev.h)
        return g1_from_abi(xy, inf.value)

    def commit_array(self, arr: np.ndarray, n=None):
        """KZG::commit (kzg.rs:61-73) from host memory: `arr` is an (n, 4) uint64
        array of Montgomery limbs (arkworks' in-memory Fr), passed to
        qg_kzg_commit as is — the drop-in path a Rust caller takes."""
        arr = np.ascontiguousarray(arr, dtype=np.uint64)
        n = arr.shape[0] if n is None else n
        xy = (C.c_uint64 * 8)()
        inf = C.c_uint8()
        check(lib().qg_kzg_commit(self.dev.h, self.h, u64p(arr), n, xy, C.byref(inf)), self.dev.h)
        return g1_from_abi(xy, inf.value)

    def msm_dev(self, vec: DeviceVec, n=None, offset: int = 0):
        """msm_unchecked(bases[offset..], vec[..n]) (qg_msm_g1_dev[_at])"""
        n = vec.n if n is None else n
        xy = (C.c_uint64 * 8)()
        inf = C.c_uint8()
        if offset:
            rc = lib().qg_msm_g1_dev_at(self.dev.h, self.h, offset, vec.h, n, xy, C.byref(inf))
        else:
            rc = lib().qg_msm_g1_dev(self.dev.h, self.h, vec.h, n, xy, C.byref(inf))
        check(rc, self.dev.h)
        return g1_from_abi(xy, inf.value)

    def msm_at(self, offset: int, scalars):
        """msm_unchecked(bases[offset..], scalars) from host scalars (qg_msm_g1_at)"""
        arr = fr_array(scalars) if len(scalars) else np.zeros((1, 4), dtype=np.uint64)
        xy = (C.c_uint64 * 8)()
        inf = C.c_uint8()
        check(lib().qg_msm_g1_at(self.dev.h, self.h, offset, u64p(arr), len(scalars), xy,
                                 C.byref(inf)), self.dev.h)
        return g1_from_abi(xy, inf.value)

    def msm_dev_batch(self, vecs, ns=None) -> list:
        """qg_msm_g1_dev_batch: the MSMs of several device vectors as one batch"""
        k = len(vecs)
        ns = [v.n for v in vecs] if ns is None else list(ns)
        hs = (C.c_void_p * max(k, 1))(*[v.h.value for v in vecs])
        nn = (C.c_size_t * max(k, 1))(*ns)
        xy = (C.c_uint64 * (8 * max(k, 1)))()
        inf = (C.c_uint8 * max(k, 1))()
        check(lib().qg_msm_g1_dev_batch(self.dev.h, self.h, hs, nn, k, xy, inf), self.dev.h)
        return [g1_from_abi(xy[8 * i:8 * i + 8], inf[i]) for i in range(k)]

    def close(self):
        if self.h:
            lib().qg_srs_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
