"""gsv — MI355X-native batch validation engine for geth-sharding's collation-validation hot path.

Host-side mirror of the reference's Go APIs for this path, over the C ABI of libgsv.so
(include/gsv.h).  Every call runs the hand-written HIP kernels for gfx950; there is no CPU
fallback (a missing libgsv.so or GPU raises).

    crypto.Ecrecover / SigToPub / Keccak256      crypto/signature_cgo.go:31-44, crypto/crypto.go:43
    types.Sender + EIP155/Homestead/Frontier     core/types/transaction_signing.go:72-247
    sharding.CalculateChunkRoot / DeriveSha      sharding/collation.go:115-119, core/types/derive_sha.go:32
    bn256.PairingCheck / precompile Run          crypto/bn256/cloudflare/bn256.go:313-327, core/vm/contracts.go:333
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading
import weakref

import numpy as np

from . import _lib
from ._lib import GsvError, check

__all__ = ["Context", "default_context", "GsvError", "device_count"]


def _np_u8(a) -> np.ndarray:
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(a), np.uint8)
    return np.ascontiguousarray(a, dtype=np.uint8)


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else None


def _pack(msgs):
    """list of bytes -> (flat uint8 array, uint64 offsets[n+1])"""
    lens = np.fromiter((len(m) for m in msgs), dtype=np.uint64, count=len(msgs))
    off = np.zeros(len(msgs) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    flat = np.frombuffer(b"".join(bytes(m) for m in msgs) + b"\0" * 8, np.uint8)
    return flat, off


def device_count() -> int:
    return int(_lib.load().gsv_device_count())


class Context:
    """One libgsv context (one HIP device): stream, HBM staging arena, precomputed tables."""

    def __init__(self, device: int = 0):
        L = _lib.load()
        h = ctypes.c_void_p()
        check(L.gsv_ctx_create(int(device), ctypes.byref(h)))
        self._h = h
        self.device = int(device)
        self._streams = []  # gsv_stream_create handles not yet destroyed
        _live.add(self)

    # -------------------------------------------------------------- lifecycle / timing
    def close(self):
        """Destroys the context and the streams it made (gsv_ctx_destroy also destroys any the caller left
        live).  Every live Context is closed at interpreter exit (atexit), before the HIP runtime's own
        static teardown, never from __del__ during module teardown."""
        if getattr(self, "_h", None):
            for q in self._streams:
                _lib.load().gsv_stream_destroy(self._h, q)
            self._streams = []
            _lib.load().gsv_ctx_destroy(self._h)
            self._h = None

    def stream_count(self):
        """(live gsv_stream_create streams, live side streams of prepared shapes)"""
        u, s = ctypes.c_int(), ctypes.c_int()
        check(_lib.load().gsv_ctx_stream_count(self._h, ctypes.byref(u), ctypes.byref(s)))
        return u.value, s.value

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_timing(self, on: bool):
        check(_lib.load().gsv_ctx_set_timing(self._h, 1 if on else 0))

    def kernel_time(self, kid: int):
        ms = ctypes.c_double()
        n = ctypes.c_long()
        check(_lib.load().gsv_ctx_kernel_time(self._h, kid, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def set_pipeline_depth(self, depth: int):
        """Instances per prepared shape from now on (gsv_ctx_set_pipeline_depth): *_dev calls of one
        shape on up to `depth` streams run concurrently."""
        check(_lib.load().gsv_ctx_set_pipeline_depth(self._h, int(depth)))

    def pipeline_streams(self, n: int):
        """`n` streams on hardware queues of their own (gsv_stream_create), as torch ExternalStreams: the
        streams of a pipeline of `n` batches (torch's pool streams can share an in-order queue, and
        batches on them then serialise).  At most _lib.MAX_STREAMS live per context."""
        import torch
        if len(self._streams) + int(n) > _lib.MAX_STREAMS:
            raise GsvError(f"{len(self._streams)} pipeline streams live, {n} more exceeds GSV_MAX_STREAMS "
                           f"({_lib.MAX_STREAMS}): destroy_streams() the previous pipeline's first")
        out = []
        for _ in range(int(n)):
            q = ctypes.c_void_p()
            check(_lib.load().gsv_stream_create(self._h, ctypes.byref(q)))
            self._streams.append(q.value)
            out.append(torch.cuda.ExternalStream(q.value, device=torch.device("cuda", self.device)))
        return out

    def destroy_streams(self, streams):
        """Destroys streams from pipeline_streams (after their work)."""
        for st in streams:
            q = int(st.cuda_stream)
            if q in self._streams:
                self._streams.remove(q)
                check(_lib.load().gsv_stream_destroy(self._h, q))

    def reset_timing(self):
        check(_lib.load().gsv_ctx_reset_timing(self._h))

    # -------------------------------------------------------------- Keccak-256
    def keccak256_batch(self, msgs) -> np.ndarray:
        n = len(msgs)
        out = np.zeros((n, 32), np.uint8)
        if n == 0:
            return out
        flat, off = _pack(msgs)
        check(_lib.load().gsv_keccak256_batch(self._h, _ptr(flat), _ptr(off), n, _ptr(out)))
        return out

    # -------------------------------------------------------------- secp256k1
    def ecrecover_batch(self, msg32, sig65, want_pub=True, want_addr=False):
        """msg32 (n,32) uint8, sig65 (n,65) uint8 -> (pub65 (n,65) | None, addr20 (n,20) | None,
        status (n,))  with ext.h / secp256.go semantics per item."""
        msg32 = np.ascontiguousarray(msg32, np.uint8).reshape(-1, 32)
        sig65 = np.ascontiguousarray(sig65, np.uint8).reshape(-1, 65)
        n = msg32.shape[0]
        if sig65.shape[0] != n:
            raise ValueError("msg32 and sig65 batch sizes differ")
        pub = np.zeros((n, 65), np.uint8) if want_pub else None
        addr = np.zeros((n, 20), np.uint8) if want_addr else None
        st = np.zeros(n, np.uint8)
        if n:
            check(_lib.load().gsv_ecrecover_batch(self._h, _ptr(msg32), _ptr(sig65), n, _ptr(pub),
                                                  _ptr(addr), _ptr(st)))
        return pub, addr, st

    def sender_batch(self, sighash32, r32, s32, v, v_big, homestead: bool):
        sighash32 = np.ascontiguousarray(sighash32, np.uint8).reshape(-1, 32)
        n = sighash32.shape[0]
        r32 = np.ascontiguousarray(r32, np.uint8).reshape(n, 32)
        s32 = np.ascontiguousarray(s32, np.uint8).reshape(n, 32)
        v = np.ascontiguousarray(v, np.uint64).reshape(n)
        v_big = np.ascontiguousarray(v_big, np.uint8).reshape(n)
        addr = np.zeros((n, 20), np.uint8)
        st = np.zeros(n, np.uint8)
        if n:
            check(_lib.load().gsv_sender_batch(self._h, _ptr(sighash32), _ptr(r32), _ptr(s32), _ptr(v),
                                               _ptr(v_big), n, 1 if homestead else 0, _ptr(addr),
                                               _ptr(st)))
        return addr, st

    def tx_sender_batch(self, txs, chain_id: int, signer_kind: int):
        n = len(txs)
        addr = np.zeros((n, 20), np.uint8)
        st = np.zeros(n, np.uint8)
        if n == 0:
            return addr, st
        flat, off = _pack(txs)
        cid = np.frombuffer(_be(chain_id) + b"\0", np.uint8)
        check(_lib.load().gsv_tx_sender_batch(self._h, _ptr(flat), _ptr(off), n, _ptr(cid),
                                              len(_be(chain_id)), int(signer_kind), _ptr(addr),
                                              _ptr(st)))
        return addr, st

    def synth_sign(self, seed: int, n: int, want_pub=True, want_addr=True):
        msg = np.zeros((n, 32), np.uint8)
        sig = np.zeros((n, 65), np.uint8)
        pub = np.zeros((n, 65), np.uint8) if want_pub else None
        addr = np.zeros((n, 20), np.uint8) if want_addr else None
        if n:
            check(_lib.load().gsv_synth_sign(self._h, ctypes.c_uint64(seed), n, _ptr(msg), _ptr(sig),
                                             _ptr(pub), _ptr(addr)))
        return msg, sig, pub, addr

    # -------------------------------------------------------------- device-resident (torch) paths
    def ecrecover_batch_dev(self, msg_t, sig_t, pub_t, addr_t, st_t, stream=None):
        """torch uint8 CUDA tensors already in HBM; enqueues on `stream` (torch stream or None)."""
        n = msg_t.shape[0]
        sp = _sp(stream)
        check(_lib.load().gsv_ecrecover_batch_dev(
            self._h, ctypes.c_void_p(msg_t.data_ptr()), ctypes.c_void_p(sig_t.data_ptr()), n,
            ctypes.c_void_p(pub_t.data_ptr()) if pub_t is not None else None,
            ctypes.c_void_p(addr_t.data_ptr()) if addr_t is not None else None,
            ctypes.c_void_p(st_t.data_ptr()), sp))

    def synth_sign_dev(self, seed, msg_t, sig_t, pub_t=None, addr_t=None, stream=None):
        n = msg_t.shape[0]
        sp = _sp(stream)
        check(_lib.load().gsv_synth_sign_dev(
            self._h, ctypes.c_uint64(seed), n, ctypes.c_void_p(msg_t.data_ptr()),
            ctypes.c_void_p(sig_t.data_ptr()),
            ctypes.c_void_p(pub_t.data_ptr()) if pub_t is not None else None,
            ctypes.c_void_p(addr_t.data_ptr()) if addr_t is not None else None, sp))

    def keccak256_batch_dev(self, data_t, off_t, out_t, stream=None):
        n = out_t.shape[0]
        sp = _sp(stream)
        check(_lib.load().gsv_keccak256_batch_dev(self._h, ctypes.c_void_p(data_t.data_ptr()),
                                                  ctypes.c_void_p(off_t.data_ptr()), n,
                                                  ctypes.c_void_p(out_t.data_ptr()), sp))


def _be(x: int) -> bytes:
    return x.to_bytes((x.bit_length() + 7) // 8, "big") if x else b""


_default = None
_default_lock = threading.Lock()
_live = weakref.WeakSet()


@atexit.register
def _close_all():
    """Interpreter exit: close every live context (its streams, shapes, communicator) while the HIP
    runtime is intact.  r05 record: a process that left CU-masked streams and the default context to
    static destructors died with SIGSEGV in __cxa_finalize after rocprofv3's finalisation
    (VERDICT r05 weak 1)."""
    global _default
    for c in list(_live):
        try:
            c.close()
        except Exception:
            pass
    _default = None


def default_context() -> Context:
    """Process-wide context on LOCAL_RANK's device (one process per GPU), created on first use,
    like the reference's global secp256k1 context (crypto/secp256k1/secp256.go:45-52)."""
    global _default
    with _default_lock:
        if _default is None:
            dev = int(os.environ.get("LOCAL_RANK", "0"))
            n = device_count()
            if n <= 0:
                raise GsvError("no HIP device visible: libgsv requires an MI355X (gfx950)")
            _default = Context(dev % n)
    return _default


def _chunk_root_batch(self, bodies) -> np.ndarray:
    """DeriveSha(Chunks(body)) for each body (sharding/collation.go:115-119)."""
    n = len(bodies)
    out = np.zeros((n, 32), np.uint8)
    if n == 0:
        return out
    flat, off = _pack(bodies)
    check(_lib.load().gsv_chunk_root_batch(self._h, _ptr(flat), _ptr(off), n, _ptr(out)))
    return out


def _chunk_root_prepare(self, h_off):
    """gsv_chunk_root_prepare: trie plans, device offset table and workspace for these offsets."""
    h_off = np.ascontiguousarray(h_off, np.uint64)
    check(_lib.load().gsv_chunk_root_prepare(self._h, _ptr(h_off), h_off.shape[0] - 1))


def _chunk_root_batch_dev(self, bodies_t, h_off, roots_t, stream=None, prepare=True):
    """bodies_t: torch uint8 CUDA tensor holding all bodies; h_off: numpy uint64 offsets (n+1).
    prepare=False skips the (idempotent, host-side) gsv_chunk_root_prepare: the call then only
    enqueues (graph-capturable) and raises GSV_E_NOT_PREPARED if the offsets were never prepared."""
    h_off = np.ascontiguousarray(h_off, np.uint64)
    n = h_off.shape[0] - 1
    if prepare:
        _chunk_root_prepare(self, h_off)
    sp = _sp(stream)
    check(_lib.load().gsv_chunk_root_batch_dev(self._h, ctypes.c_void_p(bodies_t.data_ptr()), _ptr(h_off), n,
                                               ctypes.c_void_p(roots_t.data_ptr()), sp))


def _pairing_check_batch(self, inputs) -> np.ndarray:
    """bn256Pairing precompile inputs (k x 192 bytes each) -> verdicts GSV_PAIRING_FALSE / TRUE /
    BAD_INPUT (core/vm/contracts.go:333-360, crypto/bn256/cloudflare/bn256.go:313-327)."""
    n = len(inputs)
    out = np.zeros(n, np.uint8)
    if n == 0:
        return out
    flat, off = _pack(inputs)
    check(_lib.load().gsv_bn256_pairing_check_batch(self._h, _ptr(flat), _ptr(off), n, _ptr(out)))
    return out


def _pairing_prepare(self, h_off):
    h_off = np.ascontiguousarray(h_off, np.uint64)
    check(_lib.load().gsv_bn256_pairing_prepare(self._h, _ptr(h_off), h_off.shape[0] - 1))


def _pairing_check_batch_dev(self, in_t, h_off, verdict_t, stream=None, prepare=True):
    """in_t: torch uint8 CUDA tensor with all checks; h_off: numpy uint64 offsets (n+1)."""
    h_off = np.ascontiguousarray(h_off, np.uint64)
    n = h_off.shape[0] - 1
    if prepare:
        _pairing_prepare(self, h_off)
    sp = _sp(stream)
    check(_lib.load().gsv_bn256_pairing_check_batch_dev(self._h, ctypes.c_void_p(in_t.data_ptr()), _ptr(h_off),
                                                        n, ctypes.c_void_p(verdict_t.data_ptr()), sp))


def _bn256_synth_checks_dev(self, seed, out_t, expect_t=None, stream=None):
    """configs[4] synthetic 4-pair checks into out_t (torch uint8 CUDA, nchecks x 768)."""
    n = out_t.shape[0]
    sp = _sp(stream)
    check(_lib.load().gsv_bn256_synth_checks_dev(
        self._h, ctypes.c_uint64(seed), n, ctypes.c_void_p(out_t.data_ptr()),
        ctypes.c_void_p(expect_t.data_ptr()) if expect_t is not None else None, sp))


def _sp(stream):
    """HIP stream handle for a *_dev call: None = the context's own stream.  torch's default (null)
    stream has handle 0, which the C ABI reads as "the context stream" — refused here, because the call
    would then run unordered with the caller's work on that stream."""
    if stream is None:
        return None
    h = int(stream.cuda_stream)
    if h == 0:
        raise ValueError("gsv: pass a non-default torch.cuda.Stream (or None for the context stream); "
                         "the null stream's handle 0 means the context stream in the C ABI")
    return ctypes.c_void_p(h)


def _tptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _notary_validate_shards(self, bodies, chain_id: int = 1, signer_kind: int = _lib.SIGNER_EIP155,
                            max_txs: int = 8192, want_senders=True, want_status=True):
    """Notary validation of collation bodies (gsv.h gsv_notary_validate_shards): returns
    (roots (n,32), ntx (n,), bitmap (n, ceil(max_txs/8)), senders (n,max_txs,20) | None,
    status (n,max_txs) | None)."""
    n = len(bodies)
    bm = (max_txs + 7) // 8
    roots = np.zeros((n, 32), np.uint8)
    ntx = np.zeros(n, np.uint32)
    bitmap = np.zeros((n, bm), np.uint8)
    senders = np.zeros((n, max_txs, 20), np.uint8) if want_senders else None
    status = np.zeros((n, max_txs), np.uint8) if want_status else None
    if n == 0:
        return roots, ntx, bitmap, senders, status
    flat, off = _pack(bodies)
    cid = _be(chain_id)
    cbuf = np.frombuffer(cid + b"\0", np.uint8)
    check(_lib.load().gsv_notary_validate_shards(self._h, _ptr(flat), _ptr(off), n, _ptr(cbuf), len(cid),
                                                 int(signer_kind), int(max_txs), _ptr(roots), _ptr(ntx),
                                                 _ptr(bitmap), _ptr(senders), _ptr(status)))
    return roots, ntx, bitmap, senders, status


def _notary_prepare(self, h_off, chain_id: int = 1, signer_kind: int = _lib.SIGNER_EIP155, max_txs: int = 8192):
    h_off = np.ascontiguousarray(h_off, np.uint64)
    cid = _be(chain_id)
    cbuf = np.frombuffer(cid + b"\0", np.uint8)
    check(_lib.load().gsv_notary_prepare(self._h, _ptr(h_off), h_off.shape[0] - 1, _ptr(cbuf), len(cid),
                                         int(signer_kind), int(max_txs)))


def _notary_validate_shards_dev(self, bodies_t, h_off, roots_t, ntx_t, bitmap_t, senders_t=None, status_t=None,
                                chain_id: int = 1, signer_kind: int = _lib.SIGNER_EIP155, max_txs: int = 8192,
                                stream=None, prepare=True):
    h_off = np.ascontiguousarray(h_off, np.uint64)
    n = h_off.shape[0] - 1
    if prepare:
        _notary_prepare(self, h_off, chain_id, signer_kind, max_txs)
    cid = _be(chain_id)
    cbuf = np.frombuffer(cid + b"\0", np.uint8)
    sp = _sp(stream)
    check(_lib.load().gsv_notary_validate_shards_dev(self._h, _tptr(bodies_t), _ptr(h_off), n, _ptr(cbuf), len(cid),
                                                     int(signer_kind), int(max_txs), _tptr(roots_t), _tptr(ntx_t),
                                                     _tptr(bitmap_t), _tptr(senders_t), _tptr(status_t), sp))


def _notary_synth_dev(self, seed, shard0, n_shards, txs_per_shard, bodies_t, exp_status_t=None, exp_sender_t=None,
                      stream=None):
    sp = _sp(stream)
    check(_lib.load().gsv_notary_synth_dev(self._h, ctypes.c_uint64(seed), int(shard0), int(n_shards),
                                           int(txs_per_shard), _tptr(bodies_t), _tptr(exp_status_t),
                                           _tptr(exp_sender_t), sp))


def comm_unique_id() -> bytes:
    """An RCCL unique id (gsv.h gsv_comm_unique_id): rank 0 creates it and sends it to the others."""
    buf = np.zeros(128, np.uint8)
    check(_lib.load().gsv_comm_unique_id(_ptr(buf)))
    return buf.tobytes()


def shard_range(n_shards: int, nranks: int, rank: int):
    """(first, count) of rank's contiguous shard block (gsv.h gsv_shard_range)."""
    first, count = ctypes.c_size_t(), ctypes.c_size_t()
    check(_lib.load().gsv_shard_range(n_shards, nranks, rank, ctypes.byref(first), ctypes.byref(count)))
    return first.value, count.value


def _comm_init(self, uid: bytes, nranks: int, rank: int):
    buf = np.frombuffer(bytes(uid), np.uint8).copy()
    check(_lib.load().gsv_comm_init(self._h, _ptr(buf), int(nranks), int(rank)))


def _comm_info(self):
    n, r = ctypes.c_int(), ctypes.c_int()
    check(_lib.load().gsv_comm_info(self._h, ctypes.byref(n), ctypes.byref(r)))
    return n.value, r.value


def _notary_validate_partition(self, my_bodies, n_total: int, chain_id: int = 1,
                               signer_kind: int = _lib.SIGNER_EIP155, max_txs: int = 8192,
                               want_senders=False, want_status=False):
    """gsv.h gsv_notary_validate_partition: this rank's block of bodies in, every shard's record out:
    (roots (S,32), ntx (S,), bitmap (S, ceil(max_txs/8)), senders | None, status | None) — the last
    two for this rank's shards only."""
    n = len(my_bodies)
    bm = (max_txs + 7) // 8
    roots = np.zeros((n_total, 32), np.uint8)
    ntx = np.zeros(n_total, np.uint32)
    bitmap = np.zeros((n_total, bm), np.uint8)
    senders = np.zeros((n, max_txs, 20), np.uint8) if want_senders and n else None
    status = np.zeros((n, max_txs), np.uint8) if want_status and n else None
    flat, off = _pack(my_bodies) if n else (np.zeros(1, np.uint8), np.zeros(1, np.uint64))
    cbuf = np.frombuffer(_be(chain_id) + b"\0", np.uint8)
    check(_lib.load().gsv_notary_validate_partition(self._h, _ptr(flat), _ptr(off), n_total, _ptr(cbuf),
                                                    len(_be(chain_id)), int(signer_kind), int(max_txs), _ptr(roots),
                                                    _ptr(ntx), _ptr(bitmap), _ptr(senders), _ptr(status)))
    return roots, ntx, bitmap, senders, status


def partition_block_bytes(n_total: int, nranks: int, max_txs: int = 8192) -> int:
    """Bytes of one rank's record block (gsv.h gsv_partition_block_bytes)."""
    return int(_lib.load().gsv_partition_block_bytes(n_total, nranks, max_txs))


def _notary_partition_prepare(self, h_off, n_total: int, nranks: int, rank: int, chain_id: int = 1,
                              signer_kind: int = _lib.SIGNER_EIP155, max_txs: int = 8192):
    h_off = np.ascontiguousarray(h_off, np.uint64)
    cbuf = np.frombuffer(_be(chain_id) + b"\0", np.uint8)
    check(_lib.load().gsv_notary_partition_prepare(self._h, _ptr(h_off), n_total, int(nranks), int(rank), _ptr(cbuf),
                                                   len(_be(chain_id)), int(signer_kind), int(max_txs)))


def _notary_validate_partition_dev(self, bodies_t, h_off, n_total: int, roots_t, ntx_t, bitmap_t, senders_t=None,
                                   status_t=None, rank_status_t=None, chain_id: int = 1,
                                   signer_kind: int = _lib.SIGNER_EIP155, max_txs: int = 8192, stream=None,
                                   prepare=True):
    """gsv.h gsv_notary_validate_partition_dev: this rank's block (HBM, host offsets h_off) in; every
    shard's record out in HBM (validation + pack + one ncclAllGather + unpack on `stream`)."""
    h_off = np.ascontiguousarray(h_off, np.uint64)
    if prepare:
        n, r = self.comm_info()
        _notary_partition_prepare(self, h_off, n_total, n, r, chain_id, signer_kind, max_txs)
    cbuf = np.frombuffer(_be(chain_id) + b"\0", np.uint8)
    sp = _sp(stream)
    check(_lib.load().gsv_notary_validate_partition_dev(
        self._h, _tptr(bodies_t), _ptr(h_off), n_total, _ptr(cbuf), len(_be(chain_id)), int(signer_kind),
        int(max_txs), _tptr(roots_t), _tptr(ntx_t), _tptr(bitmap_t), _tptr(senders_t), _tptr(status_t),
        _tptr(rank_status_t), sp))


def _notary_partition_pack_dev(self, bodies_t, h_off, n_total: int, nranks: int, rank: int, block_t,
                               senders_t=None, status_t=None, chain_id: int = 1,
                               signer_kind: int = _lib.SIGNER_EIP155, max_txs: int = 8192, stream=None, prepare=True):
    """gsv.h gsv_notary_partition_pack_dev: validate rank `rank`'s block and write its record block."""
    h_off = np.ascontiguousarray(h_off, np.uint64)
    if prepare:
        _notary_partition_prepare(self, h_off, n_total, nranks, rank, chain_id, signer_kind, max_txs)
    cbuf = np.frombuffer(_be(chain_id) + b"\0", np.uint8)
    sp = _sp(stream)
    check(_lib.load().gsv_notary_partition_pack_dev(
        self._h, _tptr(bodies_t), _ptr(h_off), n_total, int(nranks), int(rank), _ptr(cbuf), len(_be(chain_id)),
        int(signer_kind), int(max_txs), _tptr(block_t), _tptr(senders_t), _tptr(status_t), sp))


def _notary_partition_unpack_dev(self, blocks_t, n_total: int, nranks: int, roots_t, ntx_t, bitmap_t,
                                 rank_status_t=None, max_txs: int = 8192, stream=None):
    """gsv.h gsv_notary_partition_unpack_dev: nranks gathered blocks (rank order) -> shard-order records."""
    sp = _sp(stream)
    check(_lib.load().gsv_notary_partition_unpack_dev(self._h, _tptr(blocks_t), n_total, int(nranks), int(max_txs),
                                                      _tptr(roots_t), _tptr(ntx_t), _tptr(bitmap_t),
                                                      _tptr(rank_status_t), sp))


Context.notary_partition_prepare = _notary_partition_prepare
Context.notary_validate_partition_dev = _notary_validate_partition_dev
Context.notary_partition_pack_dev = _notary_partition_pack_dev
Context.notary_partition_unpack_dev = _notary_partition_unpack_dev
Context.comm_init = _comm_init
Context.comm_info = _comm_info
Context.notary_validate_partition = _notary_validate_partition
Context.notary_prepare = _notary_prepare
Context.chunk_root_prepare = _chunk_root_prepare
Context.pairing_prepare = _pairing_prepare
Context.notary_validate_shards = _notary_validate_shards
Context.notary_validate_shards_dev = _notary_validate_shards_dev
Context.notary_synth_dev = _notary_synth_dev
Context.bn256_synth_checks_dev = _bn256_synth_checks_dev
Context.pairing_check_batch = _pairing_check_batch
Context.pairing_check_batch_dev = _pairing_check_batch_dev
Context.chunk_root_batch = _chunk_root_batch
Context.chunk_root_batch_dev = _chunk_root_batch_dev


def _derive_sha_batch(self, lists) -> np.ndarray:
    """types.DeriveSha for each list of item RLPs (core/types/derive_sha.go:32-41): list i is a
    sequence of byte strings, item j being list.GetRlp(j) (rlp(tx) for a block's transactions)."""
    n = len(lists)
    out = np.zeros((n, 32), np.uint8)
    if n == 0:
        return out
    items = [bytes(x) for lst in lists for x in lst]
    flat, voff = _pack(items)
    list_off = np.zeros(n + 1, np.uint64)
    list_off[1:] = np.cumsum([len(lst) for lst in lists])
    check(_lib.load().gsv_derive_sha_batch(self._h, _ptr(flat), _ptr(voff), _ptr(list_off), n, _ptr(out)))
    return out


def _derive_sha_prepare(self, voff, list_off):
    voff = np.ascontiguousarray(voff, np.uint64)
    list_off = np.ascontiguousarray(list_off, np.uint64)
    check(_lib.load().gsv_derive_sha_prepare(self._h, _ptr(voff), _ptr(list_off), list_off.shape[0] - 1))


def _derive_sha_batch_dev(self, vals_t, voff, list_off, roots_t, stream=None, prepare=True):
    """vals_t: torch uint8 CUDA tensor of all item bytes; voff (items+1) / list_off (lists+1): numpy uint64."""
    voff = np.ascontiguousarray(voff, np.uint64)
    list_off = np.ascontiguousarray(list_off, np.uint64)
    n = list_off.shape[0] - 1
    if prepare:
        _derive_sha_prepare(self, voff, list_off)
    sp = _sp(stream)
    check(_lib.load().gsv_derive_sha_batch_dev(self._h, _tptr(vals_t), _ptr(voff), _ptr(list_off), n,
                                               _tptr(roots_t), sp))


def _collation_poc_batch(self, bodies, salt: bytes) -> np.ndarray:
    """Collation.CalculatePOC(salt) for each body (sharding/collation.go:124-136)."""
    n = len(bodies)
    out = np.zeros((n, 32), np.uint8)
    if n == 0:
        return out
    flat, off = _pack(bodies)
    sb = np.frombuffer(bytes(salt) + b"\0", np.uint8)
    check(_lib.load().gsv_collation_poc_batch(self._h, _ptr(flat), _ptr(off), n, _ptr(sb), len(salt), _ptr(out)))
    return out


def _collation_poc_prepare(self, h_off, salt: bytes):
    h_off = np.ascontiguousarray(h_off, np.uint64)
    sb = np.frombuffer(bytes(salt) + b"\0", np.uint8)
    check(_lib.load().gsv_collation_poc_prepare(self._h, _ptr(h_off), h_off.shape[0] - 1, _ptr(sb), len(salt)))


def _collation_poc_batch_dev(self, bodies_t, h_off, salt: bytes, out_t, stream=None, prepare=True):
    h_off = np.ascontiguousarray(h_off, np.uint64)
    n = h_off.shape[0] - 1
    if prepare:
        _collation_poc_prepare(self, h_off, salt)
    sb = np.frombuffer(bytes(salt) + b"\0", np.uint8)
    sp = _sp(stream)
    check(_lib.load().gsv_collation_poc_batch_dev(self._h, _tptr(bodies_t), _ptr(h_off), n, _ptr(sb), len(salt),
                                                  _tptr(out_t), sp))


def _collation_header_verify_batch(self, shard_id32, chunk_root32, period32, proposer20, sig65, nil_flags=None):
    """Collation header hashes + proposer-signature check (gsv.h gsv_collation_header_verify_batch):
    returns (hash32 (n,32), signer20 (n,20), status (n,))."""
    sid = _np_u8(shard_id32).reshape(-1, 32)
    n = sid.shape[0]
    root = _np_u8(chunk_root32).reshape(n, 32)
    per = _np_u8(period32).reshape(n, 32)
    prop = _np_u8(proposer20).reshape(n, 20)
    sig = _np_u8(sig65).reshape(n, 65)
    nf = None if nil_flags is None else _np_u8(nil_flags).reshape(n)
    h = np.zeros((n, 32), np.uint8)
    signer = np.zeros((n, 20), np.uint8)
    st = np.zeros(n, np.uint8)
    if n == 0:
        return h, signer, st
    check(_lib.load().gsv_collation_header_verify_batch(self._h, _ptr(sid), _ptr(root), _ptr(per), _ptr(prop),
                                                        _ptr(sig), _ptr(nf) if nf is not None else None, n,
                                                        _ptr(h), _ptr(signer), _ptr(st)))
    return h, signer, st


def _collation_header_verify_batch_dev(self, sid_t, root_t, per_t, prop_t, sig_t, st_t, nil_t=None, hash_t=None,
                                       signer_t=None, stream=None, prepare=True):
    n = sid_t.shape[0]
    if prepare:
        check(_lib.load().gsv_collation_header_prepare(self._h, n))
    sp = _sp(stream)
    check(_lib.load().gsv_collation_header_verify_batch_dev(self._h, _tptr(sid_t), _tptr(root_t), _tptr(per_t),
                                                            _tptr(prop_t), _tptr(sig_t), _tptr(nil_t), n,
                                                            _tptr(hash_t), _tptr(signer_t), _tptr(st_t), sp))


Context.collation_header_verify_batch_dev = _collation_header_verify_batch_dev
Context.derive_sha_batch = _derive_sha_batch
Context.derive_sha_batch_dev = _derive_sha_batch_dev
Context.collation_poc_batch = _collation_poc_batch
Context.collation_poc_batch_dev = _collation_poc_batch_dev
Context.collation_header_verify_batch = _collation_header_verify_batch
Context.derive_sha_prepare = _derive_sha_prepare
Context.collation_poc_prepare = _collation_poc_prepare


def _ecrecover_precompile_batch(self, inputs):
    """The ecrecover precompile's Run over many inputs (core/vm/contracts.go:78-101): returns
    (out32 (n,32), ok (n,)); ok[i] == 0 where the reference returns (nil, nil)."""
    n = len(inputs)
    out = np.zeros((n, 32), np.uint8)
    ok = np.zeros(n, np.uint8)
    if n == 0:
        return out, ok
    flat, off = _pack(inputs)
    check(_lib.load().gsv_ecrecover_precompile_batch(self._h, _ptr(flat), _ptr(off), n, _ptr(out), _ptr(ok)))
    return out, ok


def _ecrecover_precompile_batch_dev(self, in_t, out_t, ok_t, stream=None):
    """in_t: torch uint8 CUDA tensor (n, 128) of right-padded precompile inputs."""
    n = in_t.shape[0]
    sp = _sp(stream)
    check(_lib.load().gsv_ecrecover_precompile_batch_dev(self._h, _tptr(in_t), n, _tptr(out_t), _tptr(ok_t), sp))


def _prepared_shapes(self):
    cnt = ctypes.c_size_t()
    nb = ctypes.c_size_t()
    check(_lib.load().gsv_ctx_prepared_shapes(self._h, ctypes.byref(cnt), ctypes.byref(nb)))
    return cnt.value, nb.value


Context.ecrecover_precompile_batch = _ecrecover_precompile_batch
Context.ecrecover_precompile_batch_dev = _ecrecover_precompile_batch_dev
Context.prepared_shapes = _prepared_shapes
