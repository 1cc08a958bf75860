"""ctypes binding of libgsv.so (the C ABI in include/gsv.h).

The product path is the HIP library only: if libgsv.so is missing or fails to load this module
raises immediately — there is no CPU fallback anywhere in the package.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# GSV_LIB_PATH overrides the in-tree library (A/B timing of kernel variants only)
LIB_PATH = os.environ.get("GSV_LIB_PATH") or os.path.join(HERE, "libgsv.so")

# status codes (include/gsv.h)
ST_OK = 0
ST_INVALID_MSG_LEN = 1
ST_INVALID_SIG_LEN = 2
ST_INVALID_RECID = 3
ST_RECOVER_FAILED = 4
ST_INVALID_SIG = 5
ST_INVALID_CHAIN_ID = 6
ST_INVALID_PUBKEY = 7
ST_BAD_RLP = 8
ST_BN_BAD_INPUT = 9
ST_PROPOSER_MISMATCH = 10

SIGNER_EIP155 = 0
SIGNER_HOMESTEAD = 1
SIGNER_FRONTIER = 2

PAIRING_FALSE = 0
PAIRING_TRUE = 1
PAIRING_BAD_INPUT = 2

K_KECCAK = 0
K_ECRECOVER = 1
K_CHUNK_LEAF = 2
K_CHUNK_LEVEL = 3
K_PAIRING = 4
K_SENDER_PREP = 5
K_BN_PREPARE = 6
K_BN_FINAL = 7
K_NOTARY = 8
K_DERIVE_LEAF = 9
K_HEADER = 10

# API errors (negative return values)
E_INVALID_ARG = -1
E_HIP = -2
E_NOMEM = -3
E_NO_DEVICE = -4
E_TOO_LARGE = -5
E_RCCL = -6
E_NOT_PREPARED = -7

MAX_STREAMS = 8  # GSV_MAX_STREAMS: live gsv_stream_create streams per context

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t

# (name, restype, argtypes) for every symbol declared in include/gsv.h
SIGNATURES = [
    ("gsv_device_count", ctypes.c_int, []),
    ("gsv_ctx_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    ("gsv_ctx_destroy", None, [_vp]),
    ("gsv_error_string", ctypes.c_char_p, [ctypes.c_int]),
    ("gsv_abi_version", ctypes.c_int, []),
    ("gsv_ctx_set_timing", ctypes.c_int, [_vp, ctypes.c_int]),
    ("gsv_ctx_kernel_time", ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_long)]),
    ("gsv_ctx_reset_timing", ctypes.c_int, [_vp]),
    ("gsv_keccak256_batch", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp]),
    ("gsv_keccak256_batch_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _vp]),
    ("gsv_ecrecover_batch", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    ("gsv_ecrecover_batch_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    ("gsv_sender_batch", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_int, _vp, _vp]),
    ("gsv_tx_sender_batch", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, ctypes.c_int, _vp, _vp]),
    ("gsv_chunk_root_batch", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp]),
    ("gsv_chunk_root_batch_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _vp]),
    ("gsv_bn256_pairing_check_batch", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp]),
    ("gsv_bn256_pairing_check_batch_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _vp]),
    ("gsv_bn256_synth_checks_dev", ctypes.c_int, [_vp, ctypes.c_uint64, _sz, _vp, _vp, _vp]),
    ("gsv_synth_sign", ctypes.c_int, [_vp, ctypes.c_uint64, _sz, _vp, _vp, _vp, _vp]),
    ("gsv_synth_sign_dev", ctypes.c_int, [_vp, ctypes.c_uint64, _sz, _vp, _vp, _vp, _vp, _vp]),
    ("gsv_notary_validate_shards", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, ctypes.c_int, ctypes.c_uint32,
                                                  _vp, _vp, _vp, _vp, _vp]),
    ("gsv_notary_validate_shards_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, ctypes.c_int,
                                                      ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("gsv_notary_synth_dev", ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint32, _sz, ctypes.c_uint32, _vp, _vp,
                                            _vp, _vp]),
    ("gsv_derive_sha_batch", ctypes.c_int, [_vp, _vp, _vp, _vp, _sz, _vp]),
    ("gsv_derive_sha_batch_dev", ctypes.c_int, [_vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    ("gsv_collation_poc_batch", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, _vp]),
    ("gsv_collation_poc_batch_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, _vp, _vp]),
    ("gsv_collation_header_verify_batch", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    ("gsv_collation_header_verify_batch_dev", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp,
                                                             _vp]),
    ("gsv_ctx_prepared_shapes", ctypes.c_int, [_vp, ctypes.POINTER(_sz), ctypes.POINTER(_sz)]),
    ("gsv_ctx_set_pipeline_depth", ctypes.c_int, [_vp, ctypes.c_int]),
    ("gsv_stream_create", ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    ("gsv_stream_destroy", ctypes.c_int, [_vp, _vp]),
    ("gsv_ctx_stream_count", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("gsv_ecrecover_precompile_batch", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _vp]),
    ("gsv_ecrecover_precompile_batch_dev", ctypes.c_int, [_vp, _vp, _sz, _vp, _vp, _vp]),
    ("gsv_chunk_root_prepare", ctypes.c_int, [_vp, _vp, _sz]),
    ("gsv_bn256_pairing_prepare", ctypes.c_int, [_vp, _vp, _sz]),
    ("gsv_notary_prepare", ctypes.c_int, [_vp, _vp, _sz, _vp, _sz, ctypes.c_int, ctypes.c_uint32]),
    ("gsv_derive_sha_prepare", ctypes.c_int, [_vp, _vp, _vp, _sz]),
    ("gsv_collation_poc_prepare", ctypes.c_int, [_vp, _vp, _sz, _vp, _sz]),
    ("gsv_collation_header_prepare", ctypes.c_int, [_vp, _sz]),
    ("gsv_comm_unique_id", ctypes.c_int, [_vp]),
    ("gsv_comm_init", ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int]),
    ("gsv_comm_info", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("gsv_shard_range", ctypes.c_int, [_sz, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_sz), ctypes.POINTER(_sz)]),
    ("gsv_notary_validate_partition", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, ctypes.c_int, ctypes.c_uint32,
                                                     _vp, _vp, _vp, _vp, _vp]),
    ("gsv_notary_partition_prepare", ctypes.c_int, [_vp, _vp, _sz, ctypes.c_int, ctypes.c_int, _vp, _sz,
                                                    ctypes.c_int, ctypes.c_uint32]),
    ("gsv_notary_validate_partition_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, _vp, _sz, ctypes.c_int, ctypes.c_uint32,
                                                         _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("gsv_partition_block_bytes", _sz, [_sz, ctypes.c_int, ctypes.c_uint32]),
    ("gsv_notary_partition_pack_dev", ctypes.c_int, [_vp, _vp, _vp, _sz, ctypes.c_int, ctypes.c_int, _vp, _sz,
                                                     ctypes.c_int, ctypes.c_uint32, _vp, _vp, _vp, _vp]),
    ("gsv_notary_partition_unpack_dev", ctypes.c_int, [_vp, _vp, _sz, ctypes.c_int, ctypes.c_uint32, _vp, _vp, _vp,
                                                       _vp, _vp]),
]

_lib = None
_lock = threading.Lock()


class GsvError(RuntimeError):
    """A negative GSV_E_* return value from the library (`code`)."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


def load():
    """Load libgsv.so (raises OSError loudly if it is not built)."""
    global _lib
    with _lock:
        if _lib is None:
            # PyTorch-ROCm ships its own libamdhip64; when both runtimes live in one process,
            # torch's must initialise first or torch later finds no GPU.  Importing torch here (when
            # installed) makes the order independent of what the caller imported first.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            if not os.path.exists(LIB_PATH):
                raise OSError(f"libgsv.so not built at {LIB_PATH}: run `make -C geth-sharding_amd/csrc` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
            L = ctypes.CDLL(LIB_PATH)
            for name, res, args in SIGNATURES:
                f = getattr(L, name, None)
                if f is None:  # reported by tests/test_abi.py; calling it raises AttributeError
                    continue
                f.restype = res
                f.argtypes = args
            _lib = L
    return _lib


def check(rc: int):
    if rc != 0:
        msg = load().gsv_error_string(rc).decode()
        raise GsvError(f"libgsv error {rc}: {msg}", rc)
