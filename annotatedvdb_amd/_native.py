"""ctypes binding of ``libavdb_hip.so`` (the C ABI declared in ``include/avdb.h``).

The product path has exactly one implementation: the HIP kernels in this
library.  There is no CPU fallback — if the library (or a GPU) is missing,
every compute call raises :class:`NativeUnavailable`.

``torch`` is imported first on purpose: it bundles ``libamdhip64.so.7`` and the
library must bind to that same HIP runtime instance (one runtime per process),
so device pointers from torch's allocator are valid inside our kernels.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch  # noqa: F401  (loads torch's HIP runtime before ours; see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libavdb_hip.so")

ABI_VERSION = 2  # AVDB_ABI_VERSION (include/avdb.h)
AVDB_OK = 0
AVDB_EINVAL = -1
AVDB_EHIP = -2
AVDB_ENOMEM = -3
AVDB_ERANGE = -4
AVDB_ERCCL = -5
RCCL_ID_BYTES = 128

STATUS_OK = 0
STATUS_UNKNOWN_CHROM = 1
STATUS_OUT_OF_RANGE = 2
STATUS_END_BEFORE_START = 3
BIN_NONE = 0xFFFFFFFF
N_LEVELS = 14
MAX_CHROM = 64
DIGEST_CHARS = 32
MAX_PATH = 128
VCF_COUNT_WORKSPACE_BYTES = 32768  # AVDB_VCF_COUNT_WORKSPACE_BYTES (include/avdb.h)
N_COUNTERS = 32
CTR_STATUS0 = 16
CTR_RECORDS = 20
CTR_DUPLICATES = 21
CTR_HASH_COLLISIONS = 22
CTR_LONG = 23
CTR_COPY_ROWS = 24
CTR_SKIPPED_ALTS = 25
CTR_DUP_ROWS = 26
CTR_HOST_LINES = 27
CTR_EXISTING = 28
CTR_ADSP_UPDATES = 29
FORMAT_ADSP = 1
MATCH_NONE, MATCH_EXACT, MATCH_SWITCHED, MATCH_HOST = 0, 1, 2, 255
LINE_GPU, LINE_HOST, LINE_SKIP = 0, 1, 2
KEY_OK, KEY_HOST, KEY_NEED_DIGEST, KEY_OVERFLOW, KEY_DIGEST_PENDING = 0, 1, 2, 3, 4
PATH_OVERFLOW = 0x10
MAX_ALG_ID = 64


class FormatOpts(ctypes.Structure):
    """avdb_format_opts (include/avdb.h); ``struct_size`` is filled in."""
    _fields_ = [("struct_size", ctypes.c_uint32), ("max_seq_len", ctypes.c_uint32), ("alg_id", ctypes.c_char_p),
                ("flags", ctypes.c_uint32), ("match", ctypes.c_void_p), ("match_kind", ctypes.c_void_p),
                ("frag", ctypes.c_void_p), ("frag_off", ctypes.c_void_p), ("adsp_dup", ctypes.c_void_p)]

    def __init__(self, alg_id: bytes = b"", max_seq_len: int = 50, flags: int = 0):
        super().__init__(ctypes.sizeof(FormatOpts), max_seq_len, alg_id, flags)

class VcfOpts(ctypes.Structure):
    """avdb_vcf_opts (include/avdb.h); ``struct_size`` is filled in."""
    _fields_ = [("struct_size", ctypes.c_uint32), ("min_fields", ctypes.c_uint32), ("chrom_map", ctypes.c_void_p)]

    def __init__(self, min_fields: int = 0, chrom_map=None):
        super().__init__(ctypes.sizeof(VcfOpts), min_fields, chrom_map)


class LineResult(ctypes.Structure):
    """avdb_line_result (include/avdb.h)."""
    _fields_ = [(name, ctypes.c_uint32) for name in ("state", "flags", "copy_bytes", "map_bytes", "n_rec", "n_rows",
                                                     "n_skip", "n_dup", "n_upd", "reserved")]

# every symbol include/avdb.h declares (checked by tests/test_capi_symbols.py)
EXPORTED_SYMBOLS = [
    "avdb_abi_version", "avdb_last_error", "avdb_device_count",
    "avdb_ctx_create", "avdb_ctx_destroy", "avdb_ctx_n_chrom", "avdb_ctx_set_option",
    "avdb_ctx_set_sequence_digests", "avdb_l8_bin_count",
    "avdb_bin_assign", "avdb_record_prep",
    "avdb_pk_dedup_workspace_size", "avdb_pk_dedup", "avdb_pk_dedup_ex",
    "avdb_sha512t24u", "avdb_vrs_digest_workspace_size", "avdb_vrs_digest", "avdb_vrs_digest_ex",
    "avdb_format_bin_path", "avdb_format_bin_paths",
    "avdb_vcf_workspace_size", "avdb_vcf_count_workspace_size", "avdb_vcf_count_lines", "avdb_vcf_parse_lines",
    "avdb_vcf_parse_lines2", "avdb_vcf_emit", "avdb_vcf_emit_ws",
    "avdb_vcf_local_workspace_size", "avdb_vcf_parse_local", "avdb_vcf_emit_local",
    "avdb_chrom_map_create", "avdb_chrom_map_destroy",
    "avdb_format_workspace_size", "avdb_vcf_format_size", "avdb_vcf_format_write", "avdb_vcf_line_host",
    "avdb_display_attributes",
    "avdb_keyset_workspace_size", "avdb_keyset_build", "avdb_keyset_probe",
    "avdb_primary_keys", "avdb_keyset_probe_text", "avdb_primary_keys_bound",
    "avdb_primary_keys_onepass_workspace_size", "avdb_primary_keys_onepass", "avdb_primary_keys_onepass_ex",
    "avdb_primary_keys_fill_digests",
    "avdb_record_prep_keyed",
    "avdb_keyed_prep_workspace_size", "avdb_keyed_prep", "avdb_keyed_prep_lookback_errors", "avdb_vrs_digest_keys",
    "avdb_keys_off32_bytes",
    "avdb_shard_workspace_size", "avdb_vcf_select_lines", "avdb_vcf_select_copy",
    "avdb_small_prep", "avdb_small_prep_host", "avdb_bin_path_host", "avdb_annotate_host", "avdb_host_alloc", "avdb_host_free",
    "avdb_rccl_unique_id", "avdb_rccl_comm_init", "avdb_rccl_comm_destroy",
    "avdb_hist_allgather_workspace_size", "avdb_hist_allgather",
]


SMALL_PATH, SMALL_KEY, SMALL_DISPLAY = 1, 2, 4
KEYS_TOTALS_READY = 1  # AVDB_KEYS_TOTALS_READY
KEYS_DIGEST_DEFERRED = 2  # AVDB_KEYS_DIGEST_DEFERRED
KEYS_OFF32 = 4  # AVDB_KEYS_OFF32 (narrow key / path offsets)
OPT_K4_GRID, OPT_K7_GRID = 1, 2  # avdb_ctx_set_option
KEYED_TOTALS, KEYED_LONG_CODES, KEYED_DEDUP_MARKS = 1, 2, 4  # avdb_record_prep_keyed's *totals_written bits
DEDUP_MARKED = 1  # AVDB_DEDUP_MARKED
DEDUP_ONEPASS = 2  # AVDB_DEDUP_ONEPASS (marks from avdb_keyed_prep)
DIGEST_CODES_READY = 1  # AVDB_DIGEST_CODES_READY
SMALL_MAX = 65536


class SmallBatch(ctypes.Structure):
    """avdb_small_batch (include/avdb.h)."""
    _fields_ = [("chrom", ctypes.c_void_p), ("pos", ctypes.c_void_p), ("end_in", ctypes.c_void_p),
                ("allele_off", ctypes.c_void_p), ("ref_len", ctypes.c_void_p), ("alt_len", ctypes.c_void_p),
                ("heap", ctypes.c_void_p), ("ext_id", ctypes.c_void_p), ("heap_bytes", ctypes.c_size_t),
                ("n", ctypes.c_uint32), ("max_seq_len", ctypes.c_uint32), ("want", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("end_out", ctypes.c_void_p), ("code", ctypes.c_void_p),
                ("status", ctypes.c_void_p), ("key_state", ctypes.c_void_p), ("disp_state", ctypes.c_void_p),
                ("off_out", ctypes.c_void_p), ("text_out", ctypes.c_void_p * 3), ("text_cap", ctypes.c_uint32 * 3),
                ("overflow", ctypes.c_void_p)]


class NativeUnavailable(RuntimeError):
    """libavdb_hip.so (or a GPU to run it on) is not available."""


class NativeError(RuntimeError):
    def __init__(self, fn: str, rc: int, msg: str):
        super().__init__(f"{fn} failed (rc={rc}): {msg}")
        self.rc = rc


_lib = None
_lock = threading.Lock()

P = ctypes.c_void_p
SZ = ctypes.c_size_t
U32 = ctypes.c_uint32
I32 = ctypes.c_int
U8 = ctypes.c_uint8


def _sig(lib):
    f = lib
    f.avdb_abi_version.restype = I32
    f.avdb_last_error.restype = ctypes.c_char_p
    f.avdb_device_count.argtypes = [ctypes.POINTER(I32)]
    f.avdb_ctx_create.argtypes = [I32, ctypes.POINTER(U32), I32, ctypes.POINTER(P)]
    f.avdb_ctx_destroy.argtypes = [P]
    f.avdb_ctx_n_chrom.argtypes = [P]
    f.avdb_ctx_set_option.argtypes = [P, I32, ctypes.c_int64]
    f.avdb_ctx_set_sequence_digests.argtypes = [P, ctypes.c_char_p, I32]
    f.avdb_l8_bin_count.argtypes = [P, ctypes.POINTER(U32)]
    f.avdb_bin_assign.argtypes = [P, P, P, P, SZ, P, P, P, P, P]
    f.avdb_record_prep.argtypes = [P, P, P, P, P, P, P, SZ, SZ, P, P, P, P, P, P, P]
    f.avdb_pk_dedup_workspace_size.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_pk_dedup.argtypes = [P, P, P, P, P, P, P, SZ, P, SZ, I32, P, SZ, P, P, P]
    f.avdb_pk_dedup_ex.argtypes = [P, P, P, P, P, P, P, SZ, P, SZ, P, SZ, P, P, U32, P]
    f.avdb_sha512t24u.argtypes = [P, P, P, P, SZ, P, P]
    f.avdb_vrs_digest_workspace_size.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_vrs_digest.argtypes = [P, P, P, P, P, P, P, SZ, SZ, U32, P, SZ, P, P, P]
    f.avdb_vrs_digest_ex.argtypes = [P, P, P, P, P, P, P, SZ, SZ, U32, P, SZ, P, P, U32, P]
    f.avdb_format_bin_path.argtypes = [P, U8, U32, ctypes.c_char_p, SZ]
    f.avdb_format_bin_paths.argtypes = [P, P, P, SZ, P, SZ, P]
    f.avdb_vcf_workspace_size.argtypes = [SZ, SZ, ctypes.POINTER(SZ)]
    f.avdb_vcf_count_lines.argtypes = [P, P, SZ, P, SZ, P, P]
    f.avdb_vcf_parse_lines.argtypes = [P, P, SZ, SZ, P, P, SZ, P, P, P, ctypes.POINTER(VcfOpts), P]
    f.avdb_vcf_parse_lines2.argtypes = [P, P, SZ, SZ, P, SZ, P, SZ, P, P, P, ctypes.POINTER(VcfOpts), P]
    f.avdb_vcf_count_workspace_size.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_chrom_map_create.argtypes = [P, P, P, SZ, P, ctypes.POINTER(P)]
    f.avdb_chrom_map_destroy.argtypes = [P]
    f.avdb_vcf_emit.argtypes = [P, P, SZ, SZ, P, P, P, P, P, P, P, P, P, P, P, P, P]
    f.avdb_vcf_emit_ws.argtypes = [P, P, SZ, SZ, P, SZ, P, P, P, P, P, P, P, P, P, P, P, P]
    f.avdb_vcf_local_workspace_size.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_vcf_parse_local.argtypes = [P, P, SZ, P, SZ, ctypes.POINTER(VcfOpts), P, P]
    f.avdb_vcf_emit_local.argtypes = [P, P, SZ, P, SZ, P, P, P, P, P, P, P, P, P, P, P, P]
    f.avdb_format_workspace_size.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_vcf_format_size.argtypes = [P, P, SZ, SZ, P, P, P, P, P, P, P, ctypes.POINTER(FormatOpts),
                                       P, SZ, P, P, P, P]
    f.avdb_vcf_format_write.argtypes = [P, P, SZ, SZ, P, P, P, P, P, P, P, ctypes.POINTER(FormatOpts),
                                        P, P, P, P, P, P, P]
    f.avdb_vcf_line_host.argtypes = [P, ctypes.c_char_p, SZ, ctypes.POINTER(FormatOpts), ctypes.POINTER(VcfOpts), P, SZ,
                                     P, SZ, ctypes.POINTER(LineResult)]
    f.avdb_display_attributes.argtypes = [P, P, P, P, P, P, P, P, SZ, SZ, P, SZ, P, P, P, P]
    f.avdb_keyset_workspace_size.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_keyset_build.argtypes = [P, P, P, SZ, P, SZ, P]
    f.avdb_keyset_probe.argtypes = [P, P, SZ, P, P, SZ, P, P, P, P, P, P, SZ, SZ, I32, P, P, P, P]
    f.avdb_primary_keys.argtypes = [P, P, P, P, P, P, P, SZ, P, P, P, SZ, U32, P, SZ, P, P, P, SZ, P, SZ, P, P]
    f.avdb_primary_keys_onepass.argtypes = list(f.avdb_primary_keys.argtypes)  # same signature
    f.avdb_primary_keys_onepass_ex.argtypes = list(f.avdb_primary_keys.argtypes)[:-1] + [U32, P]
    f.avdb_record_prep_keyed.argtypes = list(f.avdb_record_prep.argtypes)[:-1] + [P, U32, I32, I32, P, SZ, P, SZ,
                                                                                 P, SZ, P, ctypes.POINTER(I32), P]
    f.avdb_primary_keys_fill_digests.argtypes = [P, P, P, SZ, P, P, P, P, P]
    f.avdb_keyed_prep_workspace_size.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_keyed_prep.argtypes = [P, P, P, P, P, P, P, SZ, P, SZ, U32, P, P, P, P, P, P, SZ, P, SZ, P, SZ, P,
                                  P, P, P, SZ, P, SZ, P, U32, ctypes.POINTER(I32), P]
    f.avdb_keyed_prep_lookback_errors.argtypes = [P, P, ctypes.POINTER(U32)]
    f.avdb_vrs_digest_keys.argtypes = list(f.avdb_vrs_digest_ex.argtypes)[:-1] + [P, P, P, P]
    f.avdb_keys_off32_bytes.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_primary_keys_bound.argtypes = [SZ, SZ, ctypes.POINTER(SZ), ctypes.POINTER(SZ)]
    f.avdb_primary_keys_onepass_workspace_size.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_keyset_probe_text.argtypes = [P, P, SZ, P, P, SZ, P, P, P, SZ, P, P, P]
    f.avdb_small_prep.argtypes = [P, ctypes.POINTER(SmallBatch), P]
    f.avdb_small_prep_host.argtypes = [P, ctypes.POINTER(SmallBatch)]
    f.avdb_bin_path_host.argtypes = [P, U8, U32, U32, ctypes.POINTER(U32), ctypes.POINTER(U8), P, SZ]
    f.avdb_annotate_host.argtypes = [P, ctypes.c_char_p, U32, U32, U32, I32, P, P, SZ]
    f.avdb_host_alloc.argtypes = [SZ, ctypes.POINTER(P)]
    f.avdb_host_free.argtypes = [P]
    f.avdb_shard_workspace_size.argtypes = [SZ, ctypes.POINTER(SZ)]
    f.avdb_rccl_unique_id.argtypes = [P]
    f.avdb_rccl_comm_init.argtypes = [P, I32, I32, P, ctypes.POINTER(P)]
    f.avdb_rccl_comm_destroy.argtypes = [P]
    f.avdb_hist_allgather_workspace_size.argtypes = [I32, SZ, SZ, ctypes.POINTER(SZ)]
    f.avdb_hist_allgather.argtypes = [P, P, P, SZ, P, SZ, P, P, P, SZ, P]
    f.avdb_vcf_select_lines.argtypes = [P, SZ, P, P, P, P, U32, U32, I32, P, SZ, P, P]
    f.avdb_vcf_select_copy.argtypes = [P, P, SZ, SZ, P, P, P, P]
    for name in EXPORTED_SYMBOLS:
        if name not in ("avdb_last_error",):
            getattr(f, name).restype = I32


def load_library(path: Optional[str] = None):
    """Load (once) and return the ctypes handle; raise loudly if absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("AVDB_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise NativeUnavailable(
                f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        lib = ctypes.CDLL(p)
        _sig(lib)
        if lib.avdb_abi_version() != ABI_VERSION:
            raise NativeUnavailable("libavdb_hip ABI version mismatch")
        _lib = lib
        return lib


def last_error() -> str:
    return load_library().avdb_last_error().decode(errors="replace")


def check(fn: str, rc: int) -> int:
    if rc < 0:
        raise NativeError(fn, rc, last_error())
    return rc


def ptr(t) -> int:
    """Raw device/host address of a tensor (or None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu():
    if not torch.cuda.is_available():
        raise NativeUnavailable("no ROCm GPU visible (torch.cuda.is_available() is False); "
                                "the avdb kernels run only on gfx950 — there is no CPU fallback")


_host_ctx = None


def host_ctx():
    """A process-wide context for the library's per-call host entries (K8a
    ``avdb_annotate_host`` and friends): made with device -1, so it needs no
    GPU — those entries run the kernels' record arithmetic in the library's host
    code and never launch.  Batch kernels take an ``Engine`` on a GPU."""
    global _host_ctx
    lib = load_library()
    with _lock:
        if _host_ctx is None:
            from .chromosomes import length_table
            lens = length_table("GRCh38")
            arr = (ctypes.c_uint32 * len(lens))(*lens)
            h = ctypes.c_void_p()
            rc = lib.avdb_ctx_create(-1, arr, len(lens), ctypes.byref(h))
            if rc < 0:
                raise NativeError("avdb_ctx_create", rc, lib.avdb_last_error().decode(errors="replace"))
            _host_ctx = h
        return _host_ctx
