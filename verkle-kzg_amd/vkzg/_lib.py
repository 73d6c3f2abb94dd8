"""ctypes binding of libvkzg.so (C ABI: include/vc_msm.h).

The product path: every call goes to the HIP engine. There is no CPU fallback -- if the
library is missing this raises, and on a GPU box a failing device raises too.
"""
import ctypes
import os
import re

_PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_PKG)
LIB_PATH = os.environ.get("VKZG_LIB") or os.path.join(ROOT, "lib", "libvkzg.so")
HEADERS = [os.path.join(os.path.dirname(ROOT), "include", h) for h in ("vc_msm.h", "vc_scheme.h", "vc_verkle.h",
                                                                     "vc_comm.h", "vc_group.h")]

c_void_p, c_int, c_size_t, c_uint64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64
c_double, c_long, c_char_p = ctypes.c_double, ctypes.c_long, ctypes.c_char_p
P = ctypes.c_void_p
# vc_allgather_fn (include/vc_comm.h): (user, send, bytes, recv) -> 0 on success
ALLGATHER_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_size_t, c_void_p)

SIGNATURES = {
    "vc_strerror": (c_char_p, [c_int]),
    "vc_version": (c_int, []),
    "vc_ctx_create": (c_int, [c_int, c_int, ctypes.POINTER(c_void_p)]),
    "vc_ctx_destroy": (None, [c_void_p]),
    "vc_ctx_curve": (c_int, [c_void_p]),
    "vc_ctx_set_stream": (c_int, [c_void_p, c_void_p]),
    "vc_ctx_set_option": (c_int, [c_void_p, c_int, ctypes.c_int64]),
    "vc_ctx_get_option": (c_int, [c_void_p, c_int, ctypes.POINTER(ctypes.c_int64)]),
    "vc_ctx_enable_timing": (c_int, [c_void_p, c_int]),
    "vc_ctx_kernel_time": (c_int, [c_void_p, c_char_p, ctypes.POINTER(c_double), ctypes.POINTER(c_long)]),
    "vc_ctx_reset_timing": (c_int, [c_void_p]),
    "vc_ctx_accumulate_clock": (c_int, [c_void_p, P, P]),
    "vc_host_sha256_path": (c_int, []),
    "vc_bases_upload": (c_int, [c_void_p, P, P, c_size_t, ctypes.POINTER(c_int)]),
    "vc_bases_count": (c_int, [c_void_p, c_int, ctypes.POINTER(c_size_t)]),
    "vc_bases_random": (c_int, [c_void_p, c_uint64, c_size_t, ctypes.POINTER(c_int)]),
    "vc_bases_download": (c_int, [c_void_p, c_int, P, P]),
    "vc_msm": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, P, P]),
    "vc_msm_device": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, P, P]),
    "vc_point_words": (c_int, [c_int]),
    "vc_msm_device_partial": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, P]),
    "vc_msm_partial": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, P]),
    "vc_device_mad_rate": (c_int, [c_void_p, P]),
    "vc_msm_batch_sparse": (c_int, [c_void_p, c_int, c_size_t, P, P, P, c_int, P, P]),
    "vc_verkle_new": (c_void_p, [c_int]),
    "vc_verkle_free": (None, [c_void_p]),
    "vc_verkle_insert": (c_int, [c_void_p, P, P]),
    "vc_verkle_get": (c_int, [c_void_p, P, P, P]),
    "vc_verkle_path": (c_int, [c_void_p, P, c_size_t, P, P]),
    "vc_verkle_commitment": (c_int, [c_void_p, c_int, c_void_p, P, P]),
    "vc_verkle_debug_nodes": (c_int, [c_void_p, c_size_t, P, P, P, P]),
    "vc_verkle_debug_ext_stage": (c_int, [c_void_p, c_int, P]),
    "vc_verkle_stats": (c_int, [c_void_p, P, P, P]),
    "vc_transcript_reserve": (None, [c_void_p, c_size_t]),
    "vc_msm_windows": (c_int, [c_int, c_size_t, P, P, P]),
    "vc_msm_last_plan": (c_int, [c_void_p, P, P, P, P, P]),
    "vc_msm_device_many": (c_int, [c_void_p, c_int, c_void_p, P, c_size_t, c_size_t, P, P]),
    "vc_kzg_commit_prove_device": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, P, P, P, P, P, P]),
    "vc_msm_device_window_part": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, c_int, c_int, P]),
    "vc_partials_sum": (c_int, [c_int, P, c_size_t, P, P]),
    "vc_msm_batch": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, P, P]),
    "vc_msm_batch_device": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, P, P]),
    "vc_fixed_base_precompute": (c_int, [c_void_p, c_int, c_int]),
    "vc_fixed_base_precompute_windows": (c_int, [c_void_p, c_int, c_int, c_int]),
    "vc_fixed_base_table_bytes": (c_int, [c_void_p, c_int, P]),
    "vc_fixed_base_geometry": (c_int, [c_void_p, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                       ctypes.POINTER(c_int)]),
    # vc_scheme.h
    "vc_transcript_new": (c_void_p, [c_char_p]),
    "vc_transcript_clone": (c_void_p, [c_void_p]),
    "vc_transcript_free": (None, [c_void_p]),
    "vc_transcript_append_bytes": (c_int, [c_void_p, P, c_size_t, c_char_p]),
    "vc_transcript_append_point": (c_int, [c_void_p, P, ctypes.c_uint8, c_char_p]),
    "vc_transcript_append_fr": (c_int, [c_void_p, P, c_char_p]),
    "vc_transcript_append_u64": (c_int, [c_void_p, c_uint64, c_char_p]),
    "vc_transcript_digest": (c_int, [c_void_p, c_char_p, P]),
    "vc_hash_to_field": (c_int, [P, c_size_t, P, c_size_t, P]),
    "vc_point_compress": (c_int, [P, ctypes.c_uint8, P]),
    "vc_to_data_item_batch": (c_int, [c_void_p, P, P, c_size_t, P]),
    "vc_ipa_crs": (c_int, [P, c_size_t, c_size_t, c_size_t, P]),
    "vc_kzg_setup": (c_int, [c_void_p, c_size_t, P, ctypes.POINTER(c_int), ctypes.POINTER(c_size_t)]),
    "vc_ipa_commit": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, P, P]),
    "vc_ipa_prove": (c_int, [c_void_p, c_int, c_size_t, P, P, P, P, c_size_t, P, P]),
    "vc_ipa_verify": (c_int, [c_void_p, c_int, c_size_t, P, ctypes.c_uint8, P, P, c_void_p, ctypes.POINTER(c_int)]),
    "vc_ipa_prove_commitment": (c_int, [c_void_p, c_int, c_size_t, P, P, P, c_size_t, P]),
    "vc_ipa_verify_commitment_proof": (c_int, [c_void_p, c_int, P, ctypes.c_uint8, P, ctypes.POINTER(c_int)]),
    "vc_kzg_prove": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, P, P, P, P]),
    "vc_kzg_quotient": (c_int, [c_void_p, c_size_t, P, c_size_t, P, P, P]),
    "vc_kzg_prove_all_points": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, P, P, P,
                                        ctypes.POINTER(c_size_t)]),
    "vc_kzg_prove_device": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, P, P, P, P]),
    "vc_kzg_prove_device_part": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, P, c_int, c_int, P, P]),
    "vc_multiproof_prove": (c_int, [c_void_p, c_int, c_int, c_size_t, c_size_t, P, P, P, P, P, P, P, P, P, P, P]),
    "vc_multiproof_begin": (c_int, [c_size_t, c_size_t, P, P, P, P, P, P, P]),
    "vc_multiproof_prove_many": (c_int, [c_void_p, c_int, c_int, c_size_t, c_size_t, c_size_t, c_void_p, P, P, P, P,
                                         P, P, P, P, P, P]),
    "vc_multiproof_accumulate": (c_int, [c_void_p, c_size_t, c_size_t, P, c_size_t, c_size_t, P, P, P]),
    "vc_multiproof_rows": (c_int, [c_size_t, c_size_t, P, P]),
    "vc_multiproof_begin_accumulate": (c_int, [c_void_p, c_size_t, c_size_t, P, P, P, P, c_size_t, c_size_t, P, P, P,
                                               P]),
    "vc_multiproof_finish": (c_int, [c_void_p, c_int, c_int, c_size_t, c_size_t, P, P, c_int, c_void_p, P, P, P, P,
                                     P, P]),
    "vc_multiproof_verify_ipa": (c_int, [c_void_p, c_int, c_size_t, c_size_t, P, P, P, P, P, ctypes.c_uint8, P,
                                         ctypes.POINTER(c_int)]),
    "vc_multiproof_kzg_claim": (c_int, [c_void_p, c_size_t, c_size_t, P, P, P, P, P, ctypes.c_uint8, P, P, P]),
    # vc_comm.h
    "vc_comm_unique_id": (c_int, [P]),
    "vc_comm_init_rccl": (c_int, [c_int, c_int, c_int, P, ctypes.POINTER(c_void_p)]),
    "vc_comm_init_host": (c_int, [c_int, c_int, ALLGATHER_FN, c_void_p, ctypes.POINTER(c_void_p)]),
    "vc_comm_destroy": (None, [c_void_p]),
    "vc_comm_rank": (c_int, [c_void_p]),
    "vc_comm_world": (c_int, [c_void_p]),
    "vc_comm_is_rccl": (c_int, [c_void_p]),
    "vc_comm_allgather": (c_int, [c_void_p, c_void_p, P, c_size_t, P]),
    "vc_msm_sharded": (c_int, [c_void_p, c_void_p, c_int, c_size_t, P, c_size_t, c_int, P, P]),
    "vc_msm_batch_sharded": (c_int, [c_void_p, c_void_p, c_int, c_size_t, P, c_size_t, c_int, P, P]),
    "vc_kzg_prove_sharded": (c_int, [c_void_p, c_void_p, c_int, c_size_t, P, c_size_t, P, P, P, P]),
    "vc_multiproof_prove_sharded": (c_int, [c_void_p, c_void_p, c_int, c_int, c_size_t, c_size_t, P, P, P, P, P, P,
                                            P, P, P, P, P]),
    "vc_verkle_commitment_sharded": (c_int, [c_void_p, c_void_p, c_int, c_void_p, P, P]),
    "vc_multiproof_prove_many_sharded": (c_int, [c_void_p, c_void_p, c_int, c_int, c_size_t, c_size_t, c_size_t,
                                                 c_void_p, P, P, P, P, P, P, P, P, P, P]),
    "vc_multiproof_gather": (c_int, [c_void_p, c_void_p, c_int, c_int, c_size_t, c_size_t, P, P, P, P, P, P]),
    "vc_comm_set_msm_split": (c_int, [c_void_p, c_int]),
    # vc_group.h
    "vc_group_create": (c_int, [c_int, c_int, P, ctypes.POINTER(c_void_p)]),
    "vc_group_destroy": (None, [c_void_p]),
    "vc_group_size": (c_int, [c_void_p]),
    "vc_group_peer_path": (c_int, [c_void_p, c_int, c_int]),
    "vc_group_member": (c_void_p, [c_void_p, c_int]),
    "vc_group_bases_upload": (c_int, [c_void_p, P, P, c_size_t, ctypes.POINTER(c_int)]),
    "vc_group_bases_random": (c_int, [c_void_p, c_uint64, c_size_t, ctypes.POINTER(c_int)]),
    "vc_group_kzg_setup": (c_int, [c_void_p, c_size_t, P, ctypes.POINTER(c_int), ctypes.POINTER(c_size_t)]),
    "vc_group_fixed_base_precompute": (c_int, [c_void_p, c_int, c_int, c_int]),
    "vc_group_member_table": (c_int, [c_void_p, c_int, c_int, ctypes.POINTER(c_int)]),
    "vc_group_set_msm_split": (c_int, [c_void_p, c_int]),
    "vc_group_msm": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, P, P]),
    "vc_group_msm_batch": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, c_int, P, P]),
    "vc_group_kzg_prove": (c_int, [c_void_p, c_int, c_size_t, P, c_size_t, P, P, P, P]),
    "vc_group_multiproof_prove": (c_int, [c_void_p, c_int, c_int, c_size_t, c_size_t, P, P, P, P, P, P, P, P, P, P,
                                          P]),
    "vc_group_multiproof_prove_many": (c_int, [c_void_p, c_int, c_int, c_size_t, c_size_t, c_size_t, P, P, P, P, P,
                                               P, P, P, P, P, P]),
    "vc_group_verkle_commitment": (c_int, [c_void_p, c_int, c_void_p, P, P]),
}

_lib = None


class VCError(RuntimeError):
    def __init__(self, status, where=""):
        self.status = status
        msg = lib().vc_strerror(status)
        super().__init__(f"{where}: {msg.decode() if msg else status} (status {status})")


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libvkzg.so not built at {LIB_PATH}: run `make -C verkle-kzg_amd` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7. Loading torch
        # first makes libvkzg.so bind to that copy (same soname), so engine buffers and
        # torch tensors/streams/RCCL share one runtime. Importing torch does not touch the GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status, where):
    if status != 0:
        raise VCError(status, where)


def header_functions():
    """Names of every function declared in the include/vc_*.h headers."""
    names = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(vc_[a-z0-9_]+)\s*\(", src))
    return sorted(names)
