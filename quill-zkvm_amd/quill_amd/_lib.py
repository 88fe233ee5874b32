"""ctypes binding of libquill_gpu.so (the C-ABI in include/quill_gpu.h).

The product path has no CPU fallback: if the shared library is missing or a
HIP device is unavailable, every call raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "libquill_gpu.so")

QG_OK = 0
ERRORS = {
    -1: "QG_ERR_INVALID",
    -2: "QG_ERR_DEVICE",
    -3: "QG_ERR_OOM",
    -4: "QG_ERR_UNSUPPORTED",
    -5: "QG_ERR_ASSERT",
    -6: "QG_ERR_COMM",
}


class QuillGpuError(RuntimeError):
    def __init__(self, code, msg=""):
        self.code = code
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")


class KzgOpening(C.Structure):
    _fields_ = [("x", C.c_uint64 * 4), ("y", C.c_uint64 * 4), ("proof_xy", C.c_uint64 * 8),
                ("proof_inf", C.c_uint8), ("_pad", C.c_uint8 * 7)]


class MleProof(C.Structure):
    _fields_ = [("evaluation", C.c_uint64 * 4), ("s_comm_xy", C.c_uint64 * 8),
                ("s_comm_inf", C.c_uint8), ("_pad", C.c_uint8 * 7),
                ("poly_opening", KzgOpening), ("poly_opening_inv", KzgOpening),
                ("s_opening", KzgOpening), ("s_opening_inv", KzgOpening)]


class MleOpenItem(C.Structure):
    _fields_ = [("poly", C.c_void_p), ("n", C.c_size_t), ("point", C.POINTER(C.c_uint64)),
                ("nvars", C.c_size_t), ("flags", C.c_uint32), ("_pad", C.c_uint32)]


class KzgVk(C.Structure):
    _fields_ = [("g1_xy", C.c_uint64 * 8), ("g2_xy", C.c_uint64 * 16),
                ("g2_tau_xy", C.c_uint64 * 16)]


class ExprOp(C.Structure):
    _fields_ = [("op", C.c_uint32), ("arg", C.c_uint32)]


P = C.c_void_p
U64P = C.POINTER(C.c_uint64)
U8P = C.POINTER(C.c_uint8)
U32P = C.POINTER(C.c_uint32)
SZ = C.c_size_t
# qg_challenge_fn(user, coeffs, len, out_r): the caller's transcript (qg_sumcheck_prove_cb)
CHALLENGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32,
                           C.POINTER(C.c_uint64))

# name -> (restype, argtypes)
PROTOTYPES = {
    "qg_version": (C.c_char_p, []),
    "qg_ctx_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "qg_ctx_destroy": (C.c_int, [P]),
    "qg_last_error": (C.c_char_p, [P]),
    "qg_comm_unique_id": (C.c_int, [U8P]),
    "qg_ctx_attach_comm": (C.c_int, [P, C.c_int, C.c_int, U8P]),
    "qg_loopback_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "qg_loopback_destroy": (C.c_int, [P]),
    "qg_ctx_attach_loopback": (C.c_int, [P, P, C.c_int]),
    "qg_comm_allgather_host": (C.c_int, [P, P, SZ, P]),
    "qg_comm_alltoall_host": (C.c_int, [P, P, SZ, P]),
    "qg_ctx_comm_info": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                   C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "qg_trace_full_witness": (C.c_int, [P, C.POINTER(P), C.c_uint32, C.c_uint64, P]),
    "qg_transcript_new": (C.c_int, [C.c_char_p, SZ, U8P]),
    "qg_transcript_append": (C.c_int, [U8P, C.c_char_p, SZ]),
    "qg_transcript_draw": (C.c_int, [U8P, U8P, SZ]),
    "qg_transcript_draw_fr": (C.c_int, [U8P, U64P]),
    "qg_fr_serialize": (C.c_int, [U64P, U8P]),
    "qg_g1_serialize": (C.c_int, [U64P, C.c_uint8, U8P]),
    "qg_srs_upload": (C.c_int, [P, U64P, U8P, SZ, C.POINTER(P)]),
    "qg_bases_upload": (C.c_int, [P, U64P, U8P, SZ, C.POINTER(P)]),
    "qg_srs_generate": (C.c_int, [P, U64P, U64P, SZ, C.POINTER(P)]),
    "qg_srs_generate_range": (C.c_int, [P, U64P, U64P, C.c_uint64, SZ, C.POINTER(P)]),
    "qg_srs_destroy": (C.c_int, [P]),
    "qg_srs_len": (SZ, [P]),
    "qg_srs_window_info": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "qg_srs_download": (C.c_int, [P, SZ, SZ, U64P, U8P]),
    "qg_buf_create": (C.c_int, [P, SZ, C.POINTER(P)]),
    "qg_buf_destroy": (C.c_int, [P]),
    "qg_buf_len": (SZ, [P]),
    "qg_buf_upload": (C.c_int, [P, U64P, SZ]),
    "qg_buf_download": (C.c_int, [P, U64P, SZ]),
    "qg_buf_fill_random": (C.c_int, [P, C.c_uint64]),
    "qg_buf_view": (C.c_int, [P, SZ, SZ, C.POINTER(P)]),
    "qg_buf_upload_at": (C.c_int, [P, SZ, U64P, SZ]),
    "qg_buf_upload_canonical": (C.c_int, [P, SZ, U64P, SZ]),
    "qg_buf_upload_u64": (C.c_int, [P, SZ, U64P, SZ]),
    "qg_buf_copy": (C.c_int, [P, SZ, P, SZ, SZ]),
    "qg_buf_first_mismatch": (C.c_int, [P, SZ, P, SZ, SZ, C.POINTER(C.c_int64)]),
    "qg_msm_g1": (C.c_int, [P, P, U64P, SZ, U64P, U8P]),
    "qg_msm_g1_dev": (C.c_int, [P, P, P, SZ, U64P, U8P]),
    "qg_msm_g1_at": (C.c_int, [P, P, SZ, U64P, SZ, U64P, U8P]),
    "qg_msm_g1_dev_at": (C.c_int, [P, P, SZ, P, SZ, U64P, U8P]),
    "qg_msm_g1_dev_batch": (C.c_int, [P, P, C.POINTER(P), C.POINTER(SZ), SZ,
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint8)]),
    "qg_kzg_commit": (C.c_int, [P, P, U64P, SZ, U64P, U8P]),
    "qg_kzg_open": (C.c_int, [P, P, U64P, SZ, U64P, C.POINTER(KzgOpening)]),
    "qg_mle_open": (C.c_int, [P, P, U64P, SZ, U64P, SZ, U8P, C.POINTER(MleProof)]),
    "qg_g2_generator": (C.c_int, [U64P]),
    "qg_g2_mul": (C.c_int, [U64P, C.c_uint8, U64P, U64P, U8P]),
    "qg_pairing": (C.c_int, [U64P, C.c_uint8, U64P, C.c_uint8, U64P]),
    "qg_kzg_verify": (C.c_int, [C.POINTER(KzgVk), U64P, C.c_uint8, C.POINTER(KzgOpening),
                                C.POINTER(C.c_int)]),
    "qg_mle_verify": (C.c_int, [C.POINTER(KzgVk), U64P, C.c_uint8, U64P, SZ,
                                C.POINTER(MleProof), U8P, C.POINTER(C.c_int)]),
    "qg_mle_open_dev": (C.c_int, [P, P, P, SZ, U64P, SZ, U8P, C.POINTER(MleProof)]),
    "qg_mle_open_dev_ex": (C.c_int, [P, P, P, SZ, U64P, SZ, U8P, C.c_uint32,
                                     C.POINTER(MleProof)]),
    "qg_mle_open_batch_dev": (C.c_int, [P, P, C.POINTER(MleOpenItem), SZ, U8P,
                                        C.POINTER(MleProof)]),
    "qg_eq_table": (C.c_int, [P, U64P, SZ, U64P]),
    "qg_eq_table_dev": (C.c_int, [P, U64P, SZ, P]),
    "qg_s_polynomial": (C.c_int, [P, U64P, SZ, U64P, SZ, U64P]),
    "qg_inner_product": (C.c_int, [P, U64P, SZ, U64P, SZ, U64P]),
    "qg_expr_degree": (C.c_int, [C.POINTER(ExprOp), SZ, U32P]),
    "qg_sumcheck_prove": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(U64P),
                                    C.POINTER(ExprOp), SZ, U64P, SZ, U64P, U8P, U64P, U32P,
                                    U64P, U64P]),
    "qg_sumcheck_prove_dev": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(P),
                                        C.POINTER(ExprOp), SZ, U64P, SZ, U64P, U8P, U64P, U32P,
                                        U64P, U64P]),
    "qg_sumcheck_prove_cb": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(P),
                                       C.POINTER(ExprOp), SZ, U64P, SZ, CHALLENGE_FN, P, U64P,
                                       U32P, U64P, U64P]),
    "qg_zerocheck_prove": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(U64P),
                                     C.POINTER(ExprOp), SZ, U64P, SZ, U8P, U64P, U32P, U64P,
                                     U64P, U64P]),
    "qg_zerocheck_prove_dev": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(P),
                                         C.POINTER(ExprOp), SZ, U64P, SZ, U8P, U64P, U32P,
                                         U64P, U64P]),
    "qg_logup_column": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(U64P),
                                  C.POINTER(ExprOp), SZ, U64P, SZ, C.POINTER(ExprOp), SZ, U64P,
                                  SZ, U64P, U64P, U64P]),
    "qg_logup_column_dev": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(P),
                                      C.POINTER(ExprOp), SZ, U64P, SZ, C.POINTER(ExprOp), SZ,
                                      U64P, SZ, U64P, P, U64P]),
    "qg_expr_first_nonzero_dev": (C.c_int, [P, C.c_uint32, C.c_uint32, C.POINTER(P),
                                            C.POINTER(ExprOp), SZ, U64P, SZ,
                                            C.POINTER(C.c_int64)]),
    "qg_ctx_enable_timing": (C.c_int, [P, C.c_int]),
    "qg_microbench_fq_mul": (C.c_int, [P, C.POINTER(C.c_double)]),
    "qg_selftest_inverse": (C.c_int, [P, C.c_int, C.c_int, C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64), C.c_size_t]),
    "qg_microbench_fetch": (C.c_int, [P, C.c_size_t, C.c_size_t, C.POINTER(C.c_double),
                                      C.POINTER(C.c_double)]),
    "qg_ctx_kernel_time": (C.c_int, [P, C.c_char_p, C.POINTER(C.c_double), U32P]),
    "qg_ctx_phase_split": (C.c_int, [P, C.POINTER(C.c_char_p), SZ, C.POINTER(C.c_double)]),
    "qg_trace_marker": (C.c_int, [P, C.c_uint32]),
    "qg_ctx_counter": (C.c_int, [P, C.c_char_p, C.POINTER(C.c_uint64)]),
}

_lib = None


def lib():
    """Load libquill_gpu.so (raises if it is missing: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise QuillGpuError(-2, f"{LIB_PATH} not built (run `make -C quill-zkvm_amd`)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc != QG_OK:
        msg = ""
        if ctx is not None:
            m = lib().qg_last_error(ctx)
            msg = m.decode() if m else ""
        raise QuillGpuError(rc, msg)
