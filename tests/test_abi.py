"""CPU tests of the drop-in boundary: libgsv.so loads (no GPU needed to dlopen) and exports
every symbol include/gsv.h declares, with the ctypes signatures the package binds."""
import ctypes
import os
import re

from conftest import ROOT


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "gsv.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gsv_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_boundary():
    syms = header_symbols()
    for s in ["gsv_ecrecover_batch", "gsv_sender_batch", "gsv_tx_sender_batch", "gsv_keccak256_batch",
              "gsv_chunk_root_batch", "gsv_bn256_pairing_check_batch", "gsv_notary_validate_shards"]:
        assert s in syms


def test_library_exports_every_header_symbol():
    from gsv import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_binding_covers_header():
    from gsv import _lib
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(header_symbols()) == bound


def test_no_oracle_in_product_package():
    pkg = os.path.join(ROOT, "geth-sharding_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".cuh", ".h", ".cpp")):
                txt = open(os.path.join(dp, f), errors="ignore").read()
                for bad in ("from oracle", "import oracle", "liboracle", "libgsvref", "oracle_"):
                    assert bad not in txt, (f, bad)


def test_shard_range_matches_partition_arithmetic():
    """gsv_shard_range (pure host arithmetic, callable without a GPU) == gsv/shards.py's blocks"""
    import gsv
    from gsv import shards as SH
    for n in (0, 1, 7, 100, 101):
        for world in (1, 2, 3, 8):
            got = [gsv.shard_range(n, world, r) for r in range(world)]
            want = [(SH.shard_range(r, world, n)[0], SH.shard_range(r, world, n)[1] - SH.shard_range(r, world, n)[0])
                    for r in range(world)]
            assert got == want
            assert sum(c for _, c in got) == n


def test_stream_entry_points_reject_null_arguments():
    """gsv_stream_create / gsv_stream_destroy check their arguments before any HIP call (no GPU needed)"""
    from gsv import _lib
    L = _lib.load()
    q = ctypes.c_void_p()
    assert L.gsv_stream_create(None, ctypes.byref(q)) == _lib.E_INVALID_ARG
    assert L.gsv_stream_destroy(None, None) == _lib.E_INVALID_ARG
    assert L.gsv_ctx_stream_count(None, None, None) == _lib.E_INVALID_ARG


def test_stream_cap_is_declared_and_bound():
    """GSV_MAX_STREAMS in gsv.h is the cap the package enforces (streams owned by the context)"""
    from gsv import _lib
    txt = open(os.path.join(ROOT, "include", "gsv.h")).read()
    assert int(re.search(r"#define GSV_MAX_STREAMS (\d+)", txt).group(1)) == _lib.MAX_STREAMS
    assert int(re.search(r"#define GSV_ABI_VERSION (\d+)", txt).group(1)) == _lib.load().gsv_abi_version()


def test_pipeline_streams_refuses_past_the_cap_before_any_call():
    """Context.pipeline_streams checks the cap on the Python side first, so a request past it creates
    nothing (no GPU needed: the check precedes every library call)"""
    import gsv
    import pytest
    from gsv import _lib
    c = gsv.Context.__new__(gsv.Context)
    c._h, c.device, c._streams = None, 0, [0] * (_lib.MAX_STREAMS - 1)
    with pytest.raises(gsv.GsvError):
        c.pipeline_streams(2)
