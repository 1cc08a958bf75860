"""Benchmark of the collation-validation hot path on MI355X (BASELINE.json metric:
"ecrecover sigs/sec + Keccak collation GB/s").

Default workload (BASELINE.json configs[1]): one step = recover 1,048,576 secp256k1 signatures and
derive their Keccak-256 addresses on each GPU (inputs already resident in HBM), i.e. the
crypto.Ecrecover / types.Sender hot path.  `value` = signatures recovered by all ranks / time.
Weak scaling: every rank owns its own 2^20 signatures (independent units, no data-path
collective).  The other configs are reported as legs of the same line: chunk roots (configs[2]),
notary validation with the RCCL all-gather (configs[3]), BN254 pairing checks (configs[4]), and
the §8f legs (Keccak-256 batch, tx roots, Proof of Custody, collation headers).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--legs a,b,..] [--dry-run]

--gpus N > 1 without torch.distributed's environment: bench.py starts N rank processes itself
(python -m torch.distributed.run, one per GPU, 127.0.0.1) before anything touches a GPU, and exits
with their status.  Under the driver's own launcher WORLD_SIZE must equal --gpus.  --dry-run runs
the rank setup, the shard partition, the record all-gather and the max-over-ranks timing on CPU
over gloo (no GPU, no kernels) and prints the line with "dry_run": true.
Timing: barrier + synchronize around exactly K steps, max over ranks; rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "geth-sharding_amd"))
sys.path.insert(0, ROOT)

N_SIGS = 1 << 20          # configs[1]
N_SHARDS = 100            # configs[2]/[3]
BODY = 1 << 20            # collation size limit (sharding/collation.go:45)
NOTARY_TXS = 8192         # configs[3]: 8,192 x 128-byte blob-serialized txs = one 2^20-byte body
N_CHECKS = 65536          # configs[4]: 4-pair BN254 PairingCheck x 64k (split over the ranks)
N_SENDER_CPU = 10000      # configs[0]: types.Sender over 10k EIP-155 txs on the host cores
CLOCK = 2.4e9
SIMDS = 256 * 4
# Algorithmic work per unit, REFERENCE algorithm (counted on libsecp256k1 and on the
# restatement of crypto/bn256/cloudflare): 256-bit products weighted as 8x8 = 64 (mul) / 36 (sqr)
# 32x32-bit partial products ("MAC-equivalents").
MACS_PER_RECOVERY_REF = 1358 * 64 + 1729 * 36 + 301 * 64
FP_MULS_PER_CHECK_REF = 106852            # tests/test_oracle.py pins the figure
MACS_PER_FP_MUL = 128                      # Montgomery product: 64 + 64 partial products
PERMS_PER_MIB = 83016                      # Keccak-f permutations per 1 MiB chunk root (data-independent)
# The Keccak-f[1600] instruction floor on 32-bit VALU (fixed, not the measured count, so instruction
# bloat shows in `frac`): per round, theta's column parities 2 three-input XORs per half-column (20),
# rot(C, 1) 2 v_alignbit per column (10), A ^= C[x-1] ^ rot(C[x+1]) one three-input XOR per word (50);
# rho 2 v_alignbit per rotated lane (48); chi one v_bitop3 per word (50); iota 2 v_xor: 180 per round,
# 24 rounds.  (gfx950's assembler has no v_xor3_b32: a three-input XOR is v_bitop3_b32 with table 0x96.)
KECCAK_VALU_FLOOR_PER_PERM = 24 * 180
# The same permutation priced by what each instruction costs on the SIMD (r05,
# profiles/r05/microbench_occ_ops.txt, tools/microbench_occ.hip: SIMD-cycles per wave64 instruction at
# four waves per SIMD, nominal 2.4 GHz): v_bitop3_b32 2.31 and v_xor_b32 2.37 issue at the full rate,
# v_alignbit_b32 (like every other three-source VALU op measured: v_or3, v_add3, v_bfi, v_perm,
# v_alignbyte) at half, 4.22.  The compiled round (ISA of k_chunk_level<BOTTOM>, r05 with theta applied
# as one three-input XOR per word, GSV_KECCAK_THETA3) is 120 v_bitop3 + 2 v_xor + 58 v_alignbit = the
# 180-instruction floor's count (r04: 70 + 62 + 58 with theta's D computed first), so a permutation
# holds a SIMD >= 24 x 527 cycles: the `frac_mix_ceiling` denominator, the rate a kernel doing nothing
# but this round could reach.
KECCAK_ROUND_MIX = {"v_bitop3_b32": (120, 2.31), "v_xor_b32": (2, 2.37), "v_alignbit_b32": (58, 4.22)}
KECCAK_MIX_CYCLES_PER_PERM = 24 * sum(n * c for n, c in KECCAK_ROUND_MIX.values())
# A permutation whose output is only read as a Keccak-256 digest (the sponge's last) needs state words
# 0..3 after the last round: its theta still needs all five column parities, but rho / pi / chi only the
# diagonal that lands in row 0 — 38 v_bitop3 + 2 v_xor + 18 v_alignbit = 58 instructions instead of 180
# (keccak_dev.cuh keccakf_split_digest, r06).  The floors and mix ceilings below price such a
# permutation at 23 x 180 + 58 = 4,198, so doing less than the full permutation does not read as a
# higher fraction.
KECCAK_DIGEST_ROUND_MIX = {"v_bitop3_b32": 38, "v_xor_b32": 2, "v_alignbit_b32": 18}
KECCAK_DIGEST_SAVING = 180 - sum(KECCAK_DIGEST_ROUND_MIX.values())             # 122 instructions
KECCAK_DIGEST_MIX_SAVING = sum((n - KECCAK_DIGEST_ROUND_MIX[k]) * c for k, (n, c) in KECCAK_ROUND_MIX.items())


def keccak_floor_per_perm(perms, digests):
    """Mean VALU floor per permutation of a launch with `digests` of its `perms` permutations in digest form."""
    return KECCAK_VALU_FLOOR_PER_PERM - KECCAK_DIGEST_SAVING * digests / perms


def keccak_ceiling(perms, digests):
    """Permutations/s at the instruction floor (VALU_ISSUE_PEAK wave64 instructions per SIMD-cycle)."""
    return SIMDS * VALU_ISSUE_PEAK * CLOCK * 64 / keccak_floor_per_perm(perms, digests)
# Peaks (tools/microbench_{int,lat,occ}.hip on MI355X: profiles/r01_microbench_int.txt,
# profiles/r05/microbench_occ_ops.txt):
#   VALU issue: CDNA4 SIMDs are 32 wide, a wave64 instruction issues over 2 cycles -> at most 0.5
#   wave-instructions per SIMD per cycle (MI355X_MICROARCH.md, cdna_hip_programming.md §CDNA4).
#   v_mad_u64_u32 (and every carry / 64-bit op) issues at a quarter of the 64-lane rate: 16
#   lanes/clk/SIMD = 4 cycles per wave-instruction; 4.17-4.29 measured at 2-8 waves per SIMD (r05),
#   and more waves do not raise it (k_ecrecover at 2, 3 and 4 waves/SIMD: 15.46 / 15.32 / 15.71 ms,
#   profiles/r02/ab_ecrecover_occupancy.txt, re-measured r04: profiles/r04/ab/w3_*.json).
VALU_ISSUE_PEAK = 0.5
PEAK_LANE_OPS = SIMDS * 64 * VALU_ISSUE_PEAK * CLOCK          # 7.86e13 full-rate 32-bit lane-ops/s
PEAK_MAC = SIMDS * 16 * CLOCK                                 # 3.93e13 v_mad_u64_u32 lane-ops/s
HBM_PEAK_GBPS = 8000.0
ROUND = "r06"
PROFILES = os.path.join(ROOT, "profiles", ROUND)
LEGS = ["ecrecover", "chunk_root", "notary", "keccak", "tx_root", "poc", "headers", "pairing"]


# ----------------------------------------------------------------------------- committed evidence
def _profile(name):
    try:
        with open(os.path.join(PROFILES, name)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def pmc(kernel, summary="pmc_all.json"):
    """Per-dispatch PMC figures of `kernel` from a committed rocprofv3 summary (tools/pmc_summary.py
    over tools/profile_round.sh passes); {} when absent."""
    d = _profile(summary) or {}
    return d.get(kernel, {})


def pmc_traffic(k):
    """HBM bytes per dispatch: FETCH_SIZE x 2 (gfx950 correction, MI355X_MICROARCH.md § HBM) + WRITE_SIZE."""
    if "fetch_bytes_x2" in k and "write_bytes" in k:
        return int(k["fetch_bytes_x2"] + k["write_bytes"])
    return None


def clock_fracs(units_per_launch, k, peak_units_per_s):
    """The roofline fraction from the PROFILED kernel time (k["avg_ms"], a rocprofv3 trace of the same
    leg), at the nominal 2.4 GHz peak and at the clock the profiled run held (k["profiled_clock_ghz"]:
    GRBM_GUI_ACTIVE / duration), beside the bench's own HIP-event figure."""
    if not k.get("avg_ms") or not peak_units_per_s:
        return {}
    a = units_per_launch / (k["avg_ms"] * 1e-3)
    out = {"frac_profiled_time": round(a / peak_units_per_s, 4)}
    if k.get("profiled_clock_ghz"):
        out["profiled_clock_ghz"] = k["profiled_clock_ghz"]
        out["frac_at_profiled_clock"] = round(a / (peak_units_per_s * k["profiled_clock_ghz"] * 1e9 / CLOCK), 4)
    return out


def mix_ceiling(units_per_launch, ms, digests=0):
    """The Keccak legs against the permutation's issue-cost ceiling (KECCAK_MIX_CYCLES_PER_PERM: the
    compiled round's instructions at their measured SIMD cycles; a digest permutation's last round at
    KECCAK_DIGEST_ROUND_MIX), beside the fixed instruction floor."""
    cyc = KECCAK_MIX_CYCLES_PER_PERM - KECCAK_DIGEST_MIX_SAVING * digests / units_per_launch
    peak = SIMDS * 64 * CLOCK / cyc
    out = {"mix_ceiling": round(peak / 1e9, 3), "mix_cycles_per_permutation": round(cyc),
           "mix_basis": "24 rounds x (" + " + ".join(f"{n} {k.replace('_b32', '')} x {c}" for k, (n, c) in
                                                     KECCAK_ROUND_MIX.items()) +
                        ") SIMD-cycles, profiles/r05/microbench_occ_ops.txt; a digest permutation's last "
                        "round " + " + ".join(f"{n} {k.replace('_b32', '')}" for k, n in KECCAK_DIGEST_ROUND_MIX.items())}
    if ms:
        out["frac_mix_ceiling"] = round(units_per_launch / (ms * 1e-3) / peak, 4)
    return out


def opcount(unit):
    """Field products per unit counted by the instrumented build (tools/count_ops.py ->
    profiles/<round>/opcount.json): {"mac_equiv": ..., ...} or None."""
    d = _profile("opcount.json") or {}
    return d.get(unit)


def int_lane_ops(k, ms):
    """Hardware-counted integer VALU throughput of a kernel: (SQ_INSTS_VALU_INT32 + _INT64) x 64 lanes
    per dispatch / its duration, against the full-rate lane-op peak."""
    if not k.get("sq_insts_valu_int32") or ms is None:
        return None
    ops = (k["sq_insts_valu_int32"] + k.get("sq_insts_valu_int64", 0.0)) * 64
    return {"per_launch": ops, "achieved_per_s": round(ops / (ms * 1e-3), 1), "peak_per_s": PEAK_LANE_OPS,
            "frac": round(ops / (ms * 1e-3) / PEAK_LANE_OPS, 4),
            "source": f"SQ_INSTS_VALU_INT32 + SQ_INSTS_VALU_INT64 (profiles/{ROUND}/pmc_*.json)"}


# ----------------------------------------------------------------------------- ranks
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """--gpus N > 1 outside torch.distributed.run: start N ranks as child processes (nothing in
    this process has touched a GPU) and return their exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def dist_setup(dry: bool):
    import torch
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not dry:
        torch.cuda.set_device(local)
    if ws > 1:
        import torch.distributed as dist
        if dry:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return ws, rank, local


def barrier(ws, dry=False):
    import torch
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()
    if not dry:
        torch.cuda.synchronize()


def max_over_ranks(x, ws, dry=False):
    import torch
    if ws == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if dry else "cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    # all_core runs one host thread per CPU of ONE GPU's share of the node: nproc / 8 on an 8-GPU node
    # (32 of the EPYC box's 256 threads).  The box's cgroup may cap the CPU time below that
    # (cpu.max); the quota is reported beside the thread count so the figure reads right.
    nproc = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = nproc
    return {"nproc": nproc, "cpu_model": model, "threads_all_core": max(1, nproc // 8), "affinity": affinity,
            "cgroup_cpu_quota": quota}


# ----------------------------------------------------------------------------- dry run (CPU, gloo)
def dry_run(args, ws, rank):
    """The multi-rank plumbing of the notary leg without a GPU: partition, records, gather, timing."""
    import torch
    from gsv import shards as SH
    lo, hi = SH.shard_range(rank, ws, N_SHARDS)
    per = SH.shards_per_rank(ws, N_SHARDS)
    rec = torch.zeros((per, SH.record_bytes(NOTARY_TXS)), dtype=torch.uint8)
    ids = torch.arange(lo, hi, dtype=torch.int64)
    roots = (ids.view(-1, 1) * 7 + torch.arange(32).view(1, 32)).to(torch.uint8)
    ntx = torch.full((hi - lo,), NOTARY_TXS, dtype=torch.int32)
    bm = torch.full((hi - lo, NOTARY_TXS // 8), 0xFF, dtype=torch.uint8)
    barrier(ws, dry=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        SH.pack_records(rec, roots, ntx, bm)
        g = SH.gather_records(rec, ws)
    barrier(ws, dry=True)
    dt = max_over_ranks(time.perf_counter() - t0, ws, dry=True)
    g_root, g_ntx, _ = SH.unpack_records(g, ws, N_SHARDS, NOTARY_TXS)
    assert g_root.shape[0] == N_SHARDS and bool((g_ntx == NOTARY_TXS).all())
    want = (torch.arange(N_SHARDS).view(-1, 1) * 7 + torch.arange(32).view(1, 32)).to(torch.uint8)
    assert torch.equal(g_root, want), "gathered records out of shard order"
    if rank == 0:
        print(json.dumps({
            "metric": "ecrecover sigs/sec + Keccak collation GB/s", "value": None, "unit": "sigs/s",
            "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / max(args.steps, 1) * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic", "dry_run": True,
            "config": {"workload": "dry run: rank setup + shard partition + record all-gather over gloo (no GPU)",
                       "parallelism": f"shard-partitioned x{ws}", "shards_per_rank": per,
                       "rank0_shards": [lo, hi]}}), flush=True)


# ----------------------------------------------------------------------------- CPU baselines
def _threads_run(fn, items, threads):
    """fn(item) for every item on `threads` Python threads (the work is in C: ctypes drops the GIL)."""
    it = iter(items)
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                x = next(it, None)
            if x is None:
                return
            fn(x)

    ths = [threading.Thread(target=worker) for _ in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return time.perf_counter() - t0


def cpu_ecrecover(msgs, sigs, threads):
    """The reference's libsecp256k1 recovery (oracle/_ref, geth cgo defines + ext.h), or the
    restatement when the reference build is absent.  Returns (rate, kind, pubkeys)."""
    from oracle import oracle as O
    n = msgs.shape[0]
    R = O.ref()
    kind = "reference" if R is not None else "port"
    pub = np.zeros((n, 65), np.uint8)
    u8 = ctypes.POINTER(ctypes.c_uint8)
    chunks = [(n * t // threads, n * (t + 1) // threads) for t in range(threads)]

    def run(c):
        lo, hi = c
        m = np.ascontiguousarray(msgs[lo:hi])
        s = np.ascontiguousarray(sigs[lo:hi])
        p = np.zeros((hi - lo, 65), np.uint8)
        if R is not None:
            R.gsvref_ecrecover_many(p.ctypes.data_as(u8), s.ctypes.data_as(u8), m.ctypes.data_as(u8), hi - lo)
        else:
            st = np.zeros(hi - lo, np.uint8)
            O.lib().oracle_ecrecover_batch(m.ctypes.data_as(u8), s.ctypes.data_as(u8), hi - lo,
                                           p.ctypes.data_as(u8), st.ctypes.data_as(u8), 1)
        pub[lo:hi] = p

    if R is not None:
        R.gsvref_init()
    dt = _threads_run(run, chunks, threads)
    return n / dt, kind, pub


def cpu_sender(threads_all):
    """configs[0]: types.Sender over 10,000 EIP-155 txs (chainId 1), timed as
    RLP decode + sighash RLP + Keccak + recovery + address Keccak per tx on 1 and all host threads.
    Crypto = the reference's own C (ethash sha3.c, libsecp256k1 via oracle/_ref); the RLP layer is
    the oracle's restatement of rlp/ + core/types (Go cannot run here)."""
    from oracle import cfg0
    from oracle import oracle as O
    txs, want_addr = cfg0.eip155_txs(N_SENDER_CPU)
    kind = cfg0.use_reference_crypto()
    flat = np.frombuffer(b"".join(txs) + b"\0", np.uint8)
    off = np.zeros(len(txs) + 1, np.uint64)
    off[1:] = np.cumsum([len(t) for t in txs])
    res = {}
    for label, th in (("one_core", 1), ("all_core", threads_all)):
        # repeat the 10k-tx batch until >= 1 s has passed: a shorter burst runs inside one period of
        # the box's cgroup CPU quota and reads above the sustained rate
        n_done, t_sum = 0, 0.0
        while t_sum < 1.0:
            addr, st, dt = cfg0.sender_many(flat, off, len(txs), th)
            assert (st == 0).all() and (addr == want_addr).all(), "CPU Sender disagrees with the signer"
            n_done += len(txs)
            t_sum += dt
        res[label] = round(n_done / t_sum, 1)
    O.lib().oracle_set_crypto(None, None)
    return res, kind, (txs, want_addr)


# ----------------------------------------------------------------------------- GPU legs
def leg_ecrecover(ctx, stream, dev, ws, rank, args):
    import torch
    from gsv import _lib
    msg = torch.empty((N_SIGS, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((N_SIGS, 65), dtype=torch.uint8, device=dev)
    epub = torch.empty((N_SIGS, 65), dtype=torch.uint8, device=dev)
    eaddr = torch.empty((N_SIGS, 20), dtype=torch.uint8, device=dev)
    pub = torch.empty((N_SIGS, 65), dtype=torch.uint8, device=dev)
    addr = torch.empty((N_SIGS, 20), dtype=torch.uint8, device=dev)
    st = torch.empty((N_SIGS,), dtype=torch.uint8, device=dev)
    with torch.cuda.stream(stream):
        ctx.synth_sign_dev(1000 + rank, msg, sig, epub, eaddr, stream=stream)
    stream.synchronize()

    # --ecrecover-pipeline D > 1 (2 by default since r06): consecutive batches on D streams with hardware
    # queues of their own, each with its own outputs (the recovery keeps no per-call state), so one
    # batch's last wave round overlaps the next batch's first (+1.2-1.6 % in a standalone A/B,
    # profiles/r05/ab/ecrecover_steps.txt, ecrecover_depth_live_events.txt): a node validating a stream
    # of transaction batches runs them so, as the chunk-root, notary and pairing legs do
    edepth = max(1, args.ecrecover_pipeline)
    estreams = pipeline_streams(ctx, edepth, stream, dev)
    eouts = [(pub, addr, st)] + [(torch.empty_like(pub), torch.empty_like(addr), torch.empty_like(st))
                                 for _ in range(edepth - 1)]
    for s_ in estreams:
        s_.wait_stream(stream)

    def step(i=0):
        p_, a_, s2_ = eouts[i % edepth]
        ctx.ecrecover_batch_dev(msg, sig, p_, a_, s2_, stream=estreams[i % edepth])

    for i in range(max(args.warmup, 2)):
        step(i)
    for s_ in estreams:
        s_.synchronize()
    # size-independent parity property on the full batch: recover(sign(m, d)) == pub(d), addr(d)
    for p_, a_, s2_ in eouts:
        assert int(s2_.max().item()) == 0, "recovery failed on valid signatures"
        assert torch.equal(p_, epub) and torch.equal(a_, eaddr), "recovered keys differ from signers"
    # one stream (the default): the kernel time comes from HIP events around every launch of the timed
    # region itself; batches in flight on several streams would overlap those event pairs, so there
    # it comes from a separate instrumented pass on one of the (warm) streams after the timed region
    live = edepth == 1
    if live:
        ctx.reset_timing()
        ctx.set_timing(True)
    barrier(ws)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    for s_ in estreams:
        s_.synchronize()
    barrier(ws)
    dt = max_over_ranks(time.perf_counter() - t0, ws)
    for p_, a_, s2_ in eouts:
        assert torch.equal(p_, epub) and torch.equal(a_, eaddr), "recovered keys differ from signers"
    if not live:
        ctx.reset_timing()
        ctx.set_timing(True)
        for _ in range(max(4, args.steps)):
            ctx.ecrecover_batch_dev(msg, sig, pub, addr, st, stream=estreams[0])
        estreams[0].synchronize()
    ctx.set_timing(False)
    ctx.destroy_streams(estreams)
    k_ms, k_n = ctx.kernel_time(_lib.K_ECRECOVER)
    k_avg_ms = max_over_ranks(k_ms / max(k_n, 1), ws)
    k_launches = int(k_n)
    rate = ws * N_SIGS * args.steps / dt
    k = pmc("gsv::k_ecrecover", "pmc_ecrecover.json")
    ref_ach = MACS_PER_RECOVERY_REF * N_SIGS / (k_avg_ms * 1e-3)
    oc = opcount("recovery")
    act = oc["mac_equiv"] * N_SIGS / (k_avg_ms * 1e-3) if oc else None
    roof = {"bound": "valu", "unit": "TMAC/s", "achieved": round(ref_ach / 1e12, 3), "peak": round(PEAK_MAC / 1e12, 3),
            "frac": round(ref_ach / PEAK_MAC, 4), "frac_reference_equiv": round(ref_ach / PEAK_MAC, 4),
            "frac_actual": round(act / PEAK_MAC, 4) if act else None,
            "mac_equiv_per_recovery_reference": MACS_PER_RECOVERY_REF,
            "mac_equiv_per_recovery_actual": oc["mac_equiv"] if oc else None,
            "traffic": pmc_traffic(k),
            "traffic_source": f"profiles/{ROUND}/pmc_ecrecover.json" if pmc_traffic(k) else None,
            "profiled_kernel_avg_ms": k.get("avg_ms"),
            "kernel_launches_timed": k_launches,  # the instrumented pass's launches (the last of the leg)
            "trace_agreement": f"profiles/{ROUND}/trace_agreement.json",
            "algorithmic_bytes_per_launch": N_SIGS * (32 + 65 + 65 + 20 + 1),
            # by design: one 80-byte affine comb entry per 20-bit window of u1 (13 per recovery) from the
            # 1.09 GB table in HBM (gsv_internal.h GSV_COMB_BITS)
            "comb_table_bytes_per_launch": N_SIGS * 13 * 80,
            "valu_issue_per_simd_cycle": k.get("valu_issue_per_simd_cycle"), "valu_issue_peak": VALU_ISSUE_PEAK,
            "int_lane_ops": int_lane_ops(k, k.get("avg_ms")),
            "kernel": "k_ecrecover", "kernel_avg_ms": round(k_avg_ms, 4),
            **clock_fracs(MACS_PER_RECOVERY_REF * N_SIGS, k, PEAK_MAC),
            "algorithmic_per_unit": "256-bit products as 8x8 32x32-bit partial products (mul 64, sqr 36): "
                                    f"{MACS_PER_RECOVERY_REF} per recovery for the reference algorithm "
                                    "(libsecp256k1 Strauss-wNAF), mac_equiv_per_recovery_actual = the "
                                    "v_mad_u64_u32 our kernel executes per recovery (9x29-bit fe9 products 108, "
                                    "squarings 72, dot products 189; GLV w=4 + comb; instrumented build, profiles/{ROUND}/opcount.json)".format(ROUND=ROUND)}
    state = {"msg": msg, "sig": sig, "epub": epub}
    return {"rate": rate, "dt": dt, "roofline": roof}, state


def leg_chunk_root(ctx, stream, dev, ws, rank, args):
    import torch
    from gsv import _lib
    rng = np.random.default_rng(99 + rank)
    bodies = torch.from_numpy(rng.integers(0, 256, N_SHARDS * BODY, dtype=np.uint8)).to(dev)
    h_off = np.arange(N_SHARDS + 1, dtype=np.uint64) * BODY
    # consecutive batches go to `depth` streams, each with its own instance of the prepared shape
    # (gsv_ctx_set_pipeline_depth): the latency-bound top of one batch's trie runs under the next
    # batch's leaf level, as a notary validating a stream of collations would run them
    depth = max(1, args.pipeline)
    ctx.set_pipeline_depth(depth)
    # the pipeline's streams on hardware queues of their own (gsv_stream_create): torch's pool streams
    # can share one of HIP's four in-order queues, and batches on them then serialise
    streams = pipeline_streams(ctx, depth, stream, dev)
    rootk = [torch.empty((N_SHARDS, 32), dtype=torch.uint8, device=dev) for _ in range(depth)]
    roots = rootk[0]
    ctx.chunk_root_prepare(h_off)
    ctx.set_pipeline_depth(1)
    torch.cuda.synchronize()  # the inputs were staged on torch's default stream
    csteps = max(4, args.steps)
    for i in range(max(depth, args.warmup)):
        ctx.chunk_root_batch_dev(bodies, h_off, rootk[i % depth], stream=streams[i % depth], prepare=False)
    for s_ in streams:
        s_.synchronize()
    assert all(torch.equal(r, roots) for r in rootk), "pipelined chunk roots differ between instances"
    # timed region without kernel-timing events (a step is ~10 short launches; an event pair
    # around each would add ~15 % to the step)
    barrier(ws)
    t1 = time.perf_counter()
    for i in range(csteps):
        ctx.chunk_root_batch_dev(bodies, h_off, rootk[i % depth], stream=streams[i % depth], prepare=False)
    for s_ in streams:
        s_.synchronize()
    barrier(ws)
    cdt = max_over_ranks(time.perf_counter() - t1, ws)
    ctx.destroy_streams(streams)
    # per-kernel breakdown from a separate, instrumented pass
    ctx.reset_timing()
    ctx.set_timing(True)
    for _ in range(2):
        ctx.chunk_root_batch_dev(bodies, h_off, roots, stream=stream, prepare=False)
    stream.synchronize()
    ctx.set_timing(False)
    leaf_ms, leaf_n = ctx.kernel_time(_lib.K_CHUNK_LEAF)
    lvl_ms, lvl_n = ctx.kernel_time(_lib.K_CHUNK_LEVEL)
    bot_ms = leaf_ms / max(leaf_n, 1)
    perms_step = N_SHARDS * PERMS_PER_MIB
    perms_s = ws * perms_step * csteps / cdt
    # the dominant kernel: k_chunk_level<BOTTOM>, one permutation per bottom branch node, N/16 per body
    bot_perms = N_SHARDS * BODY // 16
    k = pmc("void gsv::k_chunk_level<true>", "pmc_chunk_root.json")
    ipp = k["sq_insts_valu"] / bot_perms * 64 if k.get("sq_insts_valu") else None  # VALU instr per perm per lane
    floor = keccak_floor_per_perm(bot_perms, bot_perms)  # every bottom permutation is a digest
    ceiling = keccak_ceiling(bot_perms, bot_perms)
    traffic = pmc_traffic(k)
    bot_ach = bot_perms / (bot_ms * 1e-3)
    roof = {"bound": "valu", "unit": "Gperm/s", "kernel": "k_chunk_level<BOTTOM>", "kernel_avg_ms": round(bot_ms, 4),
            "achieved": round(bot_ach / 1e9, 3), "peak": round(ceiling / 1e9, 3) if ceiling else None,
            "frac": round(bot_ach / ceiling, 4) if ceiling else None,
            "peak_basis": f"instruction floor: {VALU_ISSUE_PEAK} wave64 VALU instructions per SIMD-cycle x 1024 "
                          f"SIMDs x 2.4 GHz x 64 lanes / {floor:.0f} VALU instructions per "
                          "permutation (the fixed Keccak-f floor, 24 x 180, with the digest permutation's last "
                          "round at 58: bench.py KECCAK_DIGEST_ROUND_MIX)",
            "valu_instr_per_permutation": round(ipp, 1) if ipp else None,
            "valu_instr_over_floor": round(ipp / floor, 3) if ipp else None,
            **clock_fracs(bot_perms, k, ceiling), **mix_ceiling(bot_perms, bot_ms, bot_perms),
            "mean_waves_per_simd": k.get("mean_waves_per_simd"),
            "valu_issue_per_simd_cycle": k.get("valu_issue_per_simd_cycle"),
            # the body bytes read + every bottom node's raw 32-byte hash written into its parent's slot
            "traffic": traffic, "algorithmic_bytes_per_launch": N_SHARDS * BODY + bot_perms * 32,
            "hbm_GBps": round(traffic / (k["avg_ms"] * 1e-3) / 1e9, 1) if traffic and k.get("avg_ms") else None,
            "hbm_frac": round(traffic / (k["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
            if traffic and k.get("avg_ms") else None,
            "permutations_per_launch": bot_perms, "profiled_kernel_avg_ms": k.get("avg_ms"),
            "trace_agreement": f"profiles/{ROUND}/trace_agreement.json"}
    out = {"collation_GBps": round(ws * N_SHARDS * BODY * csteps / cdt / 1e9, 3),
           "shards": N_SHARDS * ws, "body_bytes": BODY, "ms_per_step": round(cdt / csteps * 1e3, 3),
           "pipeline_depth": depth,
           "permutations_per_s": round(perms_s, 1),
           "bottom_kernel_avg_ms": round(bot_ms, 4),
           "level_kernels_ms_per_step": round(lvl_ms / 2, 4), "roofline": roof}
    return out, {"bodies": bodies, "roots": roots}


def _configs3_fixture():
    try:
        with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
            return json.load(f).get("configs3_notary")
    except (OSError, ValueError):
        return None


def leg_notary(ctx, stream, dev, ws, rank, args):
    """configs[3]: 100 shards x 8,192 txs partitioned by shard ID over the ranks.  Each step is the C-ABI
    call a Go notary makes (gsv_notary_validate_partition_dev): blob decode + tx RLP + Sender recovery +
    chunk root of the rank's block, the record pack, ONE ncclAllGather over the context's own RCCL
    communicator (gsv_comm_init), and the unpack into shard order on every rank."""
    import hashlib
    import torch
    from gsv import _lib
    from gsv import shards as SH
    import gsv
    lo, hi = SH.shard_range(rank, ws, N_SHARDS)
    nloc = hi - lo
    per_rank = SH.shards_per_rank(ws, N_SHARDS)
    rbytes = SH.record_bytes(NOTARY_TXS)
    nb = torch.empty((max(nloc, 1) * NOTARY_TXS * 128,), dtype=torch.uint8, device=dev)
    n_exp = torch.empty((max(nloc, 1) * NOTARY_TXS,), dtype=torch.uint8, device=dev)
    if nloc:
        ctx.notary_synth_dev(777, lo, nloc, NOTARY_TXS, nb, n_exp, None, stream=stream)
    n_off = np.arange(nloc + 1, dtype=np.uint64) * NOTARY_TXS * 128
    if ws > 1:  # the library's own communicator: rank 0 makes the RCCL id, torch.distributed carries it
        import torch.distributed as dist
        uid = [gsv.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(uid[0], ws, rank)
    a_root = torch.zeros((N_SHARDS, 32), dtype=torch.uint8, device=dev)
    a_ntx = torch.zeros((N_SHARDS,), dtype=torch.int32, device=dev)
    a_bm = torch.zeros((N_SHARDS, NOTARY_TXS // 8), dtype=torch.uint8, device=dev)
    a_rst = torch.full((ws,), -1, dtype=torch.int32, device=dev)
    n_st = torch.empty((max(nloc, 1), NOTARY_TXS), dtype=torch.uint8, device=dev)
    stream.wait_stream(torch.cuda.current_stream())  # the fills above ran on torch's stream
    # consecutive collation batches kept in flight on `depth` streams (shape instances): one step's
    # validation overlaps the previous step's tail and all-gather; the library orders the all-gathers
    # on its communicator.  A rank's block at N = 8 (13 shards) is 1.6k waves, less than one round of
    # the GPU's 2,048 wave slots, so one step alone leaves it partly idle (tools/notary_sweep.py)
    depth = max(1, args.notary_pipeline)
    ctx.set_pipeline_depth(depth)
    ctx.notary_partition_prepare(n_off, N_SHARDS, ws, rank, max_txs=NOTARY_TXS)
    ctx.set_pipeline_depth(1)
    n_streams = pipeline_streams(ctx, depth, stream, dev)  # on queues of their own (as the chunk-root leg)
    outs = [(a_root, a_ntx, a_bm, a_rst)] + [(torch.zeros_like(a_root), torch.zeros_like(a_ntx), torch.zeros_like(a_bm),
                                             torch.full_like(a_rst, -1)) for _ in range(depth - 1)]
    for s_ in n_streams:
        s_.wait_stream(torch.cuda.current_stream())
        s_.wait_stream(stream)

    def notary_step(with_status=False, i=0):
        r_, c_, b_, st_ = outs[i % depth]
        ctx.notary_validate_partition_dev(nb, n_off, N_SHARDS, r_, c_, b_, None,
                                          n_st if with_status else None, st_, max_txs=NOTARY_TXS,
                                          stream=n_streams[i % depth], prepare=False)

    notary_step(with_status=True)
    n_streams[0].synchronize()
    # full-size parity: every tx status of this rank's block equals the construction, and the gathered
    # records of all 100 shards equal the committed configs[3] fixture (oracle/_ref + restatement)
    assert int(a_rst.min()) == 0 and int(a_rst.max()) == 0, f"rank statuses {a_rst.tolist()}"
    if nloc:
        assert torch.equal(n_st.view(-1)[:nloc * NOTARY_TXS], n_exp[:nloc * NOTARY_TXS]), \
            "notary statuses differ from the constructed truth"
    assert bool((a_ntx == NOTARY_TXS).all())
    fx = _configs3_fixture()
    fixture_ok = None
    if fx is not None and fx["seed"] == 777 and fx["shards"] == N_SHARDS:
        got = [bytes(r).hex() for r in a_root.cpu().numpy()]
        assert got == fx["roots"], "gathered chunk roots differ from the configs[3] fixture"
        assert hashlib.sha256(a_bm.cpu().numpy().tobytes()).hexdigest() == fx["bitmaps_sha256"], \
            "gathered validity bitmaps differ from the configs[3] fixture"
        fixture_ok = True
    # cross-check of the collective: the same records through torch.distributed (RCCL) agree
    t_root = torch.zeros((max(nloc, 1), 32), dtype=torch.uint8, device=dev)
    t_cnt = torch.zeros((max(nloc, 1),), dtype=torch.int32, device=dev)
    t_bm = torch.zeros((max(nloc, 1), NOTARY_TXS // 8), dtype=torch.uint8, device=dev)
    stream.wait_stream(torch.cuda.current_stream())
    if nloc:
        ctx.notary_validate_shards_dev(nb, n_off, t_root, t_cnt, t_bm, None, None, max_txs=NOTARY_TXS,
                                       stream=stream)
    rec = torch.zeros((per_rank, rbytes), dtype=torch.uint8, device=dev)
    with torch.cuda.stream(stream):
        SH.pack_records(rec, t_root[:nloc], t_cnt[:nloc], t_bm[:nloc])
        gathered = SH.gather_records(rec, ws)
    stream.synchronize()
    g_root, g_ntx, g_bm = SH.unpack_records(gathered, ws, N_SHARDS, NOTARY_TXS)
    assert torch.equal(g_root, a_root) and torch.equal(g_ntx, a_ntx) and torch.equal(g_bm, a_bm), \
        "C-ABI RCCL records differ from the torch.distributed gather"
    # Strong scaling: a rank's step shrinks with N (13 of the 100 shards at N = 8), so each rank times N
    # times the steps and the timed region spans about the same wall time at every N.  A pipeline's
    # fill and drain cost about one step's latency (~1.3 ms at 13 shards) per timed region: 12 timed
    # 13-shard steps read 1.28 ms per step, 40 read 1.16 (the steady state; 100 shards 8.76 ms, i.e.
    # 98 % of linear), profiles/r06/ab/notary_stagger_steps.txt.  --steps of them per rank at N = 1 (r05:
    # --steps / 2), as the ecrecover and chunk-root legs
    nsteps = max(2 * depth, args.steps) * ws
    for i in range(1, max(depth, args.warmup)):  # warm the other instances (at least --warmup steps)
        notary_step(i=i)
    for s_ in n_streams:
        s_.synchronize()
    barrier(ws)
    t4 = time.perf_counter()
    for i in range(nsteps):
        notary_step(i=i)
    for s_ in n_streams:
        s_.synchronize()
    barrier(ws)
    ndt = max_over_ranks(time.perf_counter() - t4, ws)
    for r_, c_, b_, st_ in outs:  # every instance's last gathered records equal the checked ones
        assert torch.equal(r_, a_root) and torch.equal(c_, a_ntx) and torch.equal(b_, a_bm)
        assert int(st_.min()) == 0 and int(st_.max()) == 0
    ctx.reset_timing()  # kernel breakdown from a separate, instrumented step
    ctx.set_timing(True)
    notary_step()
    n_streams[0].synchronize()
    ctx.set_timing(False)
    ctx.destroy_streams(n_streams)
    k_not, _ = ctx.kernel_time(_lib.K_NOTARY)
    assert int(a_rst.max()) == 0
    # roofline of the rank's step: the recovery's v_mad_u64_u32 (opcount notary_tx,
    # per tx) plus the Keccak-f permutations (the chunk roots' PERMS_PER_MIB per 1 MiB body, the sighash
    # and address of every tx: one each for these <= 135-byte strings), both priced at their VALU peak
    # and summed as SIMD time; the permutations are converted to MAC-equivalents at the two peaks' ratio
    oc = opcount("notary_tx")
    roof = None
    if oc:
        ntx = nloc * NOTARY_TXS
        perms = nloc * PERMS_PER_MIB + 2 * ntx
        # digest permutations counted: the bottom branch nodes (N / 16 per body); the chunk roots' other
        # hashed nodes (< 4,400 per MiB) are priced at the full floor
        perm_peak = keccak_ceiling(perms, nloc * BODY // 16)
        mac_eq = oc["mac_equiv"] * ntx + perms * PEAK_MAC / perm_peak
        kt = pmc("gsv::k_notary_tx", "pmc_notary.json")
        kb = pmc("gsv::k_blob_index", "pmc_notary.json")
        tx_work = (oc["mac_equiv"] + 2 * PEAK_MAC / perm_peak) * ntx  # what k_notary_tx does
        roof = {"bound": "valu", "unit": "TMAC/s", "scope": "the rank's whole step (ms_per_step)",
                "achieved": round(mac_eq / (ndt / nsteps) / 1e12, 3), "peak": round(PEAK_MAC / 1e12, 3),
                "frac": round(mac_eq / (ndt / nsteps) / PEAK_MAC, 4),
                "work_per_step": {"txs": ntx, "mac_per_tx": oc["mac_equiv"], "permutations": perms,
                                  "mac_equiv_per_permutation": round(PEAK_MAC / perm_peak, 1),
                                  "mac_equiv": round(mac_eq)},
                "basis": "v_mad_u64_u32 of k_notary_tx (profiles/{R}/opcount.json notary_tx) + Keccak-f "
                         "permutations at the fixed instruction floor (bench.py keccak_floor_per_perm), as SIMD "
                         "time at the 2.4 GHz VALU peaks".format(R=ROUND),
                "tx_kernels_frac": round(tx_work / (k_not * 1e-3) / PEAK_MAC, 4) if k_not else None,
                "k_notary_tx": {"profiled_avg_ms": kt.get("avg_ms"),
                                "frac_profiled_time": round(tx_work / (kt["avg_ms"] * 1e-3) / PEAK_MAC, 4)
                                if kt.get("avg_ms") and nloc == N_SHARDS else None,
                                "profiled_clock_ghz": kt.get("profiled_clock_ghz"),
                                "valu_issue_per_simd_cycle": kt.get("valu_issue_per_simd_cycle"),
                                "mean_waves_per_simd": kt.get("mean_waves_per_simd"),
                                "scratch_bytes_per_lane": kt.get("scratch_bytes_per_lane"),
                                "traffic": pmc_traffic(kt), "write_bytes": kt.get("write_bytes")},
                "k_blob_index_profiled_avg_ms": kb.get("avg_ms"),
                "source": "profiles/{R}/pmc_notary.json: leg-only passes with no side streams "
                          "(GSV_MAX_SIDE_STREAMS=0), overlapped dispatches dropped".format(R=ROUND)}
    out = {"shards_per_s": round(N_SHARDS * nsteps / ndt, 2),
           "txs_per_s": round(N_SHARDS * NOTARY_TXS * nsteps / ndt, 1),
           "shards": N_SHARDS, "txs_per_shard": NOTARY_TXS, "shards_per_rank": per_rank,
           "ms_per_step": round(ndt / nsteps * 1e3, 3), "tx_kernels_ms_per_step": round(k_not, 3),
           "pipeline_depth": depth,
           "entry_point": "gsv_notary_validate_partition_dev (C ABI)",
           "collective": "ncclAllGather on the library's RCCL communicator (gsv_comm_init)" if ws > 1
           else "none (1 rank: the block is copied)",
           "collective_cross_check": "torch.distributed all_gather_into_tensor (RCCL) of the same records: equal"
           if ws > 1 else "local",
           "fixture_configs3": "100 roots + bitmap digest equal tests/golden/configs.json" if fixture_ok
           else "fixture absent",
           "gathered_bytes_per_step": ws * gsv.partition_block_bytes(N_SHARDS, ws, NOTARY_TXS),
           "scaling": "strong", "roofline": roof}
    return out, {"nb": nb, "n_exp": n_exp, "n_root": a_root[lo:hi] if nloc else a_root[:0]}


def _tx_strings(rank):
    # 2,000 blocks x 200 RLP strings of 100-160 bytes (random bytes: the trie and the sponge only see
    # the item strings)
    rng = np.random.default_rng(11 + rank)
    nblk, ntx = 2000, 200
    lens = rng.integers(100, 161, nblk * ntx).astype(np.uint64)
    voff = np.zeros(nblk * ntx + 1, np.uint64)
    np.cumsum(lens, out=voff[1:])
    vals = rng.integers(0, 256, int(voff[-1]), dtype=np.uint8)
    return nblk, ntx, lens, voff, vals


def leg_keccak(ctx, stream, dev, ws, rank, args):
    """crypto.Keccak256 over 400,000 tx RLP strings (the tx-hash / sighash workload, A10): one
    message per lane, offsets and data resident in HBM."""
    import torch
    from gsv import _lib
    nblk, ntx, lens, voff, vals_np = _tx_strings(rank)
    vals = torch.from_numpy(vals_np).to(dev)
    koff_t = torch.from_numpy(voff.astype(np.int64)).to(dev)
    kout = torch.empty((nblk * ntx, 32), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # the inputs were staged on torch's default stream
    ctx.keccak256_batch_dev(vals, koff_t, kout, stream=stream)
    stream.synchronize()
    # consecutive batches on two streams with hardware queues of their own (the batch call keeps no
    # per-call state, so two run at once into two output buffers): one 0.1-ms launch's ramp-up and tail
    # overlap the next one's; 40 timed batches (r04 timed 5 on one stream: 0.5 ms, launch-latency noise)
    kdepth = max(1, args.pipeline)  # (as the chunk-root leg; the leg-only profile passes run 1)
    kstreams = pipeline_streams(ctx, kdepth, stream, dev)
    kouts = [kout] + [torch.empty_like(kout) for _ in range(kdepth - 1)]
    for s_ in kstreams:
        s_.wait_stream(stream)
    ksteps = 40
    for i in range(4):  # warm-up on every stream
        ctx.keccak256_batch_dev(vals, koff_t, kouts[i % kdepth], stream=kstreams[i % kdepth])
    for s_ in kstreams:
        s_.synchronize()
    barrier(ws)
    t8 = time.perf_counter()
    for i in range(ksteps):
        ctx.keccak256_batch_dev(vals, koff_t, kouts[i % kdepth], stream=kstreams[i % kdepth])
    for s_ in kstreams:
        s_.synchronize()
    barrier(ws)
    kdt = max_over_ranks(time.perf_counter() - t8, ws)
    assert all(torch.equal(kouts[0], o) for o in kouts), "keccak256 batch results differ between the streams"
    ctx.destroy_streams(kstreams)
    ctx.reset_timing()
    ctx.set_timing(True)
    # ten one-at-a-time launches for the per-launch figure: a 0.1-ms kernel's first launch on the leg's
    # own stream after the pipeline read up to 10 % long over two (r06 trace agreement 1.11)
    for _ in range(10):
        ctx.keccak256_batch_dev(vals, koff_t, kout, stream=stream)
    stream.synchronize()
    ctx.set_timing(False)
    k_ms, k_n = ctx.kernel_time(_lib.K_KECCAK)
    kavg = k_ms / max(k_n, 1)
    if rank == 0 and not args.no_cpu_baseline:  # sample vs the oracle sponge
        from oracle import oracle as O
        hv = vals_np[:int(voff[64])].tobytes()
        ko = kout[:64].cpu().numpy()
        assert all(bytes(ko[i]) == O.keccak256(hv[int(voff[i]):int(voff[i + 1])]) for i in range(64)), \
            "keccak256 batch mismatch vs oracle"
    perms = int(np.sum(lens // 136 + 1))
    k = pmc("gsv::k_keccak256", "pmc_keccak.json")
    ipp = k["sq_insts_valu"] / perms * 64 if k.get("sq_insts_valu") else None
    nmsg = nblk * ntx  # one digest permutation per message
    floor = keccak_floor_per_perm(perms, nmsg)
    ceiling = keccak_ceiling(perms, nmsg)
    ach = perms / (kavg * 1e-3)
    traffic = pmc_traffic(k)
    roof = {"bound": "valu", "unit": "Gperm/s", "kernel": "k_keccak256", "kernel_avg_ms": round(kavg, 4),
            "achieved": round(ach / 1e9, 3), "peak": round(ceiling / 1e9, 3) if ceiling else None,
            "frac": round(ach / ceiling, 4) if ceiling else None,
            "peak_basis": "instruction floor (as chunk_root.roofline: the fixed Keccak-f floor of "
                          f"{KECCAK_VALU_FLOOR_PER_PERM} VALU instructions per permutation, a message's digest "
                          f"permutation at {KECCAK_VALU_FLOOR_PER_PERM - KECCAK_DIGEST_SAVING}: {floor:.0f} on average)",
            "valu_instr_per_permutation": round(ipp, 1) if ipp else None,
            "valu_instr_over_floor": round(ipp / floor, 3) if ipp else None,
            **clock_fracs(perms, k, ceiling), **mix_ceiling(perms, kavg, nmsg),
            "mean_waves_per_simd": k.get("mean_waves_per_simd"),
            "valu_issue_per_simd_cycle": k.get("valu_issue_per_simd_cycle"),
            "traffic": traffic, "algorithmic_bytes_per_launch": int(voff[-1]) + (nblk * ntx + 1) * 8 + nblk * ntx * 32,
            "hbm_GBps": round(traffic / (k["avg_ms"] * 1e-3) / 1e9, 1) if traffic and k.get("avg_ms") else None,
            "permutations_per_launch": perms, "profiled_kernel_avg_ms": k.get("avg_ms"),
            # the same against the pipelined throughput (two batches in flight): launch ramp-up and
            # tail overlapped with the neighbouring batch
            "frac_pipelined": round(perms * ksteps / kdt / ceiling, 4) if ceiling else None}
    return {"hashes_per_s": round(ws * nblk * ntx * ksteps / kdt, 1),
            "GBps": round(ws * float(voff[-1]) * ksteps / kdt / 1e9, 3),
            "permutations_per_s": round(ws * perms * ksteps / kdt, 1),
            "messages": nblk * ntx, "bytes_per_message": "100-160",
            "ms_per_step": round(kdt / ksteps * 1e3, 3), "pipeline_depth": kdepth, "roofline": roof}


def leg_tx_root(ctx, stream, dev, ws, rank, args):
    """DeriveSha(block.Transactions()) (core/block_validator.go:70) over 2,000 blocks x 200 txs."""
    import torch
    nblk, ntx, lens, voff, vals_np = _tx_strings(rank)
    vals = torch.from_numpy(vals_np).to(dev)
    list_off = np.arange(nblk + 1, dtype=np.uint64) * ntx
    # consecutive batches on --pipeline streams with their own shape instances (as the chunk-root leg):
    # one batch's latency-bound trie heights run beside the next batch's leaf hashing
    tdepth = max(1, args.pipeline)
    ctx.set_pipeline_depth(tdepth)
    ctx.derive_sha_prepare(voff, list_off)
    ctx.set_pipeline_depth(1)
    tstreams = pipeline_streams(ctx, tdepth, stream, dev)
    trk = [torch.empty((nblk, 32), dtype=torch.uint8, device=dev) for _ in range(tdepth)]
    troots = trk[0]
    torch.cuda.synchronize()  # the inputs were staged on torch's default stream
    for i in range(tdepth):
        ctx.derive_sha_batch_dev(vals, voff, list_off, trk[i], stream=tstreams[i], prepare=False)
    for s_ in tstreams:
        s_.synchronize()
    assert all(torch.equal(r, troots) for r in trk), "pipelined tx roots differ between instances"
    tsteps = 20  # (r04: 3 steps, a 1.3-ms timed region)
    barrier(ws)
    t5 = time.perf_counter()
    for i in range(tsteps):
        ctx.derive_sha_batch_dev(vals, voff, list_off, trk[i % tdepth], stream=tstreams[i % tdepth], prepare=False)
    for s_ in tstreams:
        s_.synchronize()
    barrier(ws)
    tdt = max_over_ranks(time.perf_counter() - t5, ws)
    ctx.destroy_streams(tstreams)
    if rank == 0 and not args.no_cpu_baseline:
        from oracle import oracle as O
        items = [vals_np[int(voff[j]):int(voff[j + 1])].tobytes() for j in range(ntx)]
        assert bytes(troots[0].cpu().numpy()) == O.derive_sha(items), "tx root mismatch vs oracle"
    return {"blocks_per_s": round(ws * nblk * tsteps / tdt, 1), "txs_per_s": round(ws * nblk * ntx * tsteps / tdt, 1),
            "MBps_of_tx_rlp": round(ws * float(voff[-1]) * tsteps / tdt / 1e6, 1),
            "blocks": nblk, "txs_per_block": ntx, "ms_per_step": round(tdt / tsteps * 1e3, 3),
            "pipeline_depth": tdepth}


def leg_poc(ctx, stream, dev, ws, rank, args):
    """Proof of Custody (sharding/collation.go:124-136): 100 x 1 MiB bodies, 20-byte salt
    (sharding/collation_test.go:318) -> 21 MiB salted chunk tries."""
    import torch
    prng = np.random.default_rng(13 + rank)
    pbodies = torch.from_numpy(prng.integers(0, 256, N_SHARDS * BODY, dtype=np.uint8)).to(dev)
    p_off = np.arange(N_SHARDS + 1, dtype=np.uint64) * BODY
    salt = bytes(range(1, 21))
    # consecutive batches on --pipeline streams with their own shape instances (each holds its 2.1 GB of
    # salted bodies): one batch's expansion and trie top run beside the other batch's leaf level
    qdepth = max(1, args.pipeline)
    ctx.set_pipeline_depth(qdepth)
    ctx.collation_poc_prepare(p_off, salt)
    ctx.set_pipeline_depth(1)
    qstreams = pipeline_streams(ctx, qdepth, stream, dev)
    pk = [torch.empty((N_SHARDS, 32), dtype=torch.uint8, device=dev) for _ in range(qdepth)]
    pocs = pk[0]
    torch.cuda.synchronize()  # the inputs were staged on torch's default stream
    for i in range(qdepth):
        ctx.collation_poc_batch_dev(pbodies, p_off, salt, pk[i], stream=qstreams[i], prepare=False)
    for s_ in qstreams:
        s_.synchronize()
    assert all(torch.equal(r, pocs) for r in pk), "pipelined POC roots differ between instances"
    qsteps = 2 * qdepth
    barrier(ws)
    t6 = time.perf_counter()
    for i in range(qsteps):
        ctx.collation_poc_batch_dev(pbodies, p_off, salt, pk[i % qdepth], stream=qstreams[i % qdepth], prepare=False)
    for s_ in qstreams:
        s_.synchronize()
    barrier(ws)
    qdt = max_over_ranks(time.perf_counter() - t6, ws)
    ctx.destroy_streams(qstreams)
    return {"bodies_per_s": round(ws * N_SHARDS * qsteps / qdt, 2),
            "body_GBps": round(ws * N_SHARDS * BODY * qsteps / qdt / 1e9, 3),
            "salted_GBps": round(ws * N_SHARDS * BODY * 21 * qsteps / qdt / 1e9, 3),
            "salt_bytes": 20, "ms_per_step": round(qdt / qsteps * 1e3, 3), "pipeline_depth": qdepth}


def leg_headers(ctx, stream, dev, ws, rank, args, sig):
    """Collation header hash + proposer signature: 2^20 headers with random fields and valid ECDSA
    signatures over other messages -> every status GSV_ST_PROPOSER_MISMATCH (same work as a match)."""
    import torch
    from gsv import _lib
    nh = 1 << 20
    hsid = torch.randint(0, 256, (nh, 32), dtype=torch.uint8, device=dev)
    hroot = torch.randint(0, 256, (nh, 32), dtype=torch.uint8, device=dev)
    hper = torch.randint(0, 256, (nh, 32), dtype=torch.uint8, device=dev)
    hprop = torch.randint(0, 256, (nh, 20), dtype=torch.uint8, device=dev)
    hst = torch.empty((nh,), dtype=torch.uint8, device=dev)
    hhash = torch.empty((nh, 32), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # the inputs were staged on torch's default stream
    # consecutive batches in flight on dedicated-queue streams (--ecrecover-pipeline, as the recovery leg;
    # the shape prepared at that depth, one instance per stream): one batch's header hashes and compare
    # run beside the other batch's recovery
    hdepth = max(1, args.ecrecover_pipeline)
    ctx.set_pipeline_depth(hdepth)
    ctx.collation_header_verify_batch_dev(hsid, hroot, hper, hprop, sig, hst, None, hhash, None, stream=stream)
    ctx.set_pipeline_depth(1)
    stream.synchronize()
    assert bool((hst == _lib.ST_PROPOSER_MISMATCH).all()), "header signatures failed to recover"
    hstreams = pipeline_streams(ctx, hdepth, stream, dev)
    houts = [(hst, hhash)] + [(torch.empty_like(hst), torch.empty_like(hhash)) for _ in range(hdepth - 1)]
    for s_ in hstreams:
        s_.wait_stream(stream)

    def hstep(i):
        st_, h_ = houts[i % hdepth]
        ctx.collation_header_verify_batch_dev(hsid, hroot, hper, hprop, sig, st_, None, h_, None,
                                              stream=hstreams[i % hdepth], prepare=False)

    for i in range(hdepth):
        hstep(i)
    for s_ in hstreams:
        s_.synchronize()
    assert all(torch.equal(st_, hst) and torch.equal(h_, hhash) for st_, h_ in houts), \
        "pipelined header results differ between instances"
    hsteps = 3 * hdepth
    barrier(ws)
    t7 = time.perf_counter()
    for i in range(hsteps):
        hstep(i)
    for s_ in hstreams:
        s_.synchronize()
    barrier(ws)
    hdt = max_over_ranks(time.perf_counter() - t7, ws)
    ctx.destroy_streams(hstreams)
    return {"headers_per_s": round(ws * nh * hsteps / hdt, 1), "headers": nh, "ms_per_step": round(hdt / hsteps * 1e3, 3),
            "batches_in_flight": hdepth}


def pipeline_streams(ctx, depth, stream, dev):
    """The streams a leg's pipeline spreads consecutive batches over: on hardware queues of their own
    (gsv_stream_create); GSV_BENCH_TORCH_STREAMS=1 takes the leg's stream and torch pool streams instead
    (A/B: those can share one of HIP's four in-order queues)."""
    import torch
    if os.environ.get("GSV_BENCH_TORCH_STREAMS") != "1":
        try:
            return ctx.pipeline_streams(depth)
        except Exception as e:  # a box whose HIP refuses CU-masked streams: still measure, say so
            print(f"bench: gsv_stream_create failed ({e}); pipelines on torch streams", file=sys.stderr)
    return [stream] + [torch.cuda.Stream(device=dev) for _ in range(depth - 1)]


def leg_pairing(ctx, stream, dev, ws, rank, args):
    import torch
    from gsv import _lib
    nloc = N_CHECKS // ws + (1 if rank < N_CHECKS % ws else 0)
    if args.pairing_checks:  # one GPU standing in for a rank of an N-GPU run (8,192 = N = 8)
        nloc = args.pairing_checks
    pin = torch.empty((nloc, 768), dtype=torch.uint8, device=dev)
    pexp = torch.empty((nloc,), dtype=torch.uint8, device=dev)
    pver = torch.empty((nloc,), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()  # the inputs were staged on torch's default stream
    ctx.bn256_synth_checks_dev(5000 + rank, pin, pexp, stream=stream)
    p_off = np.arange(nloc + 1, dtype=np.uint64) * 768
    stream.synchronize()
    # consecutive batches on `depth` streams with their own shape instances (as the chunk-root leg):
    # one batch's latency-bound Miller / final-exponentiation waves share the SIMDs with the next
    # batch's kernels.  auto: one at 65,536 checks and up, where every kernel alone fills the GPU and
    # overlapping batches only contend (r05, streams on queues of their own: 19.56 / 20.57 / 20.56 /
    # 20.20 ms per batch at depth 1-4, profiles/r05/ab/pairing_depth_dedicated.txt); six below, where
    # the library then takes the work-efficient layout (k = 4, one-lane final: 8,192 checks 3.13 ms per
    # batch against 3.30 at r05's depth 4, r06, profiles/r06/ab/pairing_rank_depth.txt)
    depth = args.pairing_pipeline if args.pairing_pipeline > 0 else (6 if nloc < 65536 else 1)
    ctx.set_pipeline_depth(depth)
    streams = pipeline_streams(ctx, depth, stream, dev)  # on queues of their own (as the chunk-root leg)
    pvk = [pver] + [torch.empty_like(pver) for _ in range(depth - 1)]
    ctx.pairing_prepare(p_off)
    ctx.set_pipeline_depth(1)
    for i in range(max(depth, args.warmup)):  # warm-up (every stream, at least --warmup batches)
        ctx.pairing_check_batch_dev(pin, p_off, pvk[i % depth], stream=streams[i % depth], prepare=False)
    for s_ in streams:
        s_.synchronize()
    # size-independent parity property at full size: every verdict equals the generator's
    assert all(torch.equal(v, pexp) for v in pvk), "pairing verdicts differ from the constructed truth"
    # small per-rank batches: enough batches that the pipeline's fill and drain (about one batch
    # latency, depth x the per-batch time) stay a small part of the timed region
    # (strong scaling, as the notary leg: N times the batches at N ranks, about the same wall time)
    psteps = max((6 if depth <= 3 else 2 * depth) if nloc >= 65536 else 6 * depth, args.steps // 2) * ws
    barrier(ws)
    t2 = time.perf_counter()
    for i in range(psteps):
        ctx.pairing_check_batch_dev(pin, p_off, pvk[i % depth], stream=streams[i % depth], prepare=False)
    for s_ in streams:
        s_.synchronize()
    barrier(ws)
    pdt = max_over_ranks(time.perf_counter() - t2, ws)
    ctx.destroy_streams(streams)
    assert all(torch.equal(v, pexp) for v in pvk), "pairing verdicts differ from the constructed truth"
    # per-kernel breakdown from a separate, instrumented single-stream pass
    ctx.reset_timing()
    ctx.set_timing(True)
    isteps = min(psteps, 24)  # the breakdown needs a few launches, not the timed region's N x count
    for _ in range(isteps):
        ctx.pairing_check_batch_dev(pin, p_off, pver, stream=stream, prepare=False)
    stream.synchronize()
    ctx.set_timing(False)
    k_prep, _ = ctx.kernel_time(_lib.K_BN_PREPARE)
    k_mill, _ = ctx.kernel_time(_lib.K_PAIRING)
    k_fin, _ = ctx.kernel_time(_lib.K_BN_FINAL)
    k_tot = (k_prep + k_mill + k_fin) / isteps
    oc = opcount("pairing_check")
    act = oc["mac_equiv"] * nloc / (k_tot * 1e-3) if oc else None
    kk = {n: pmc(f"gsv::bn::{n}", "pmc_pairing.json") for n in ("k_bn_lines", "k_bn_miller", "k_bn_final")}
    if not kk["k_bn_lines"]:  # the two-wave lines kernel (large batches, r05)
        kk["k_bn_lines"] = pmc("gsv::bn::k_bn_lines_w2", "pmc_pairing.json")
    # headline = the v_mad_u64_u32 our kernels execute (frac_actual).  The reference algorithm's work
    # (its 254-bit Order*Q subgroup check included, which this path replaces by three psi maps on the
    # line chain's final point) is reported only as a work ratio, not as a roofline fraction
    k_prof = sum(v.get("avg_ms") or 0.0 for v in kk.values())
    roof = {"bound": "valu", "unit": "TMAC/s", "achieved": round(act / 1e12, 3) if act else None,
            "peak": round(PEAK_MAC / 1e12, 3), "frac": round(act / PEAK_MAC, 4) if act else None,
            "frac_actual": round(act / PEAK_MAC, 4) if act else None,
            **(clock_fracs(oc["mac_equiv"] * nloc, {"avg_ms": k_prof,
                                                    "profiled_clock_ghz": kk["k_bn_miller"].get("profiled_clock_ghz")},
                           PEAK_MAC) if oc and k_prof and nloc == N_CHECKS else {}),
            "reference_work_ratio": round(FP_MULS_PER_CHECK_REF * MACS_PER_FP_MUL / oc["mac_equiv"], 3) if oc else None,
            "mac_equiv_per_check_reference": FP_MULS_PER_CHECK_REF * MACS_PER_FP_MUL,
            "mac_equiv_per_check_actual": oc["mac_equiv"] if oc else None,
            "fp_products_per_check_actual": oc.get("fp_products") if oc else None,
            "kernels_ms_per_step": round(k_tot, 3),
            "per_kernel": {n: {"valu_issue_per_simd_cycle": v.get("valu_issue_per_simd_cycle"),
                               "traffic": pmc_traffic(v),
                               # rocprofv3's vgpr_count as recorded; on gfx950 it reads half the ISA's
                               # VGPR + AGPR allocation (k_bn_final 256 for 256 + 256, k_ecrecover 120
                               # for 234; DESIGN.md §3.4 lists the ISA figures)
                               "rocprof_vgpr_count": v.get("vgpr"),
                               "scratch_bytes_per_lane": v.get("scratch_bytes_per_lane")} for n, v in kk.items()},
            "algorithmic_per_unit": f"{FP_MULS_PER_CHECK_REF} F_p Montgomery products x {MACS_PER_FP_MUL} partial "
                                    "products per 4-pair check for the reference algorithm (its 254-bit Order*Q "
                                    "subgroup check included); mac_equiv_per_check_actual = the v_mad_u64_u32 our "
                                    "kernels execute per check (9x29-bit F_p products 81 + Montgomery reductions 81; "
                                    "psi subgroup test, precomputed lines, multi-Miller loop; instrumented build, "
                                    "profiles/{ROUND}/opcount.json)".format(ROUND=ROUND)}
    total = nloc * ws if args.pairing_checks else N_CHECKS
    out = {"checks_per_s": round(total * psteps / pdt, 1), "checks": total, "checks_per_rank": nloc,
           "pipeline_depth": depth,
           "pairs_per_check": 4, "roofline": roof, "ms_per_step": round(pdt / psteps * 1e3, 3),
           "prepare_kernel_ms": round(k_prep / isteps, 3), "miller_kernel_ms": round(k_mill / isteps, 3),
           "final_exp_kernel_ms": round(k_fin / isteps, 3),
           "verdicts": {"true": int((pexp == 1).sum().item()), "false": int((pexp == 0).sum().item()),
                        "bad_input": int((pexp == 2).sum().item())}}
    return out, {"pin": pin, "pexp": pexp}


# ----------------------------------------------------------------------------- CPU legs (rank 0, N = 1)
def cpu_baselines(ctx, legs, st, res, info):
    """every leg's CPU side on the box's host cores, one core and all cores
    (`threads_all_core` = one GPU's share of an 8-GPU node, nproc / 8 threads; the box's cgroup CPU
    quota is reported beside it).  Bounded samples of the same workloads."""
    from oracle import oracle as O
    th = info["threads_all_core"]
    out = {}
    ec = st.get("ecrecover")
    if ec is not None:
        sample1, sampleN = 4096, 4096 * th
        m_h = ec["msg"][:sampleN].cpu().numpy()
        s_h = ec["sig"][:sampleN].cpu().numpy()
        r1, kind, p1 = cpu_ecrecover(m_h[:sample1], s_h[:sample1], 1)
        rN, _, pN = cpu_ecrecover(m_h, s_h, th)
        assert (pN == ec["epub"][:sampleN].cpu().numpy()).all(), "CPU baseline disagrees with the GPU"
        out["ecrecover"] = {"one_core": round(r1, 1), "all_core": round(rN, 1), "unit": "sigs/s", "kind": kind,
                            "sample": f"{sample1} (1 core) / {sampleN} ({th} threads) signatures of the configs[1] "
                                      "workload, libsecp256k1 secp256k1_ext_ecdsa_recover (oracle/_ref)"}
    sres, skind, (txs, want) = cpu_sender(th)
    out["sender"] = dict(sres, unit="txs/s", kind=skind,
                         sample=f"configs[0]: types.Sender over {N_SENDER_CPU} EIP-155 txs (chainId 1), RLP "
                                "(oracle restatement) + Keccak (ethash sha3.c) + recovery (libsecp256k1)")
    # the same 10k txs through the GPU's types.Sender (host-pointer path, PCIe-inclusive)
    flat = np.frombuffer(b"".join(txs) + b"\0", np.uint8)
    t0 = time.perf_counter()
    gaddr, gst = ctx.tx_sender_batch(txs, 1, 0)
    gdt = time.perf_counter() - t0
    assert (gst == 0).all() and (gaddr == want).all(), "GPU Sender disagrees with the CPU path"
    out["sender"]["gpu_host_path_txs_per_s"] = round(len(txs) / gdt, 1)
    del flat
    if "chunk_root" in st:
        cb = st["chunk_root"]["bodies"]
        nbd = min(N_SHARDS, 2 * th)  # two bodies per thread: >= 1 s of sustained work
        bodies = [cb[i * BODY:(i + 1) * BODY].cpu().numpy().tobytes() for i in range(nbd)]
        roots = [None] * nbd
        t1 = _threads_run(lambda i: roots.__setitem__(i, O.derive_sha_bytes(bodies[i])), [0], 1)
        tN = _threads_run(lambda i: roots.__setitem__(i, O.derive_sha_bytes(bodies[i])), list(range(nbd)), th)
        gr = st["chunk_root"]["roots"][:nbd].cpu().numpy()
        assert all(roots[i] == bytes(gr[i]) for i in range(nbd)), "chunk root mismatch vs oracle"
        out["chunk_root"] = {"one_core": round(BODY / t1 / 1e9, 4), "all_core": round(nbd * BODY / tN / 1e9, 4),
                             "unit": "GB/s of collation body", "kind": "port",
                             "sample": f"1 body (1 thread) / {nbd} bodies ({th} threads) of 1 MiB, oracle DeriveSha "
                                       "restatement"}
    if "notary" in st:
        from oracle import cfg0
        cfg0.use_reference_crypto()
        nb = st["notary"]["nb"]
        nshard = min(th, nb.shape[0] // (NOTARY_TXS * 128))
        bodies = [nb[i * NOTARY_TXS * 128:(i + 1) * NOTARY_TXS * 128].cpu().numpy().tobytes() for i in range(nshard)]
        stats = [None] * nshard

        def shard(i):
            blobs = O.blob_deserialize(bodies[i])
            tx = [b for b, _ in blobs]
            fl = np.frombuffer(b"".join(tx) + b"\0", np.uint8)
            of = np.zeros(len(tx) + 1, np.uint64)
            of[1:] = np.cumsum([len(x) for x in tx])
            _, s, _ = cfg0.sender_many(fl, of, len(tx), 1)
            stats[i] = (s, O.derive_sha_bytes(bodies[i]))

        t1 = _threads_run(shard, [0], 1)
        tN = _threads_run(shard, list(range(nshard)), th)
        O.lib().oracle_set_crypto(None, None)
        exp = st["notary"]["n_exp"][:NOTARY_TXS].cpu().numpy()
        assert (stats[0][0] == exp).all(), "notary statuses vs CPU path"
        assert stats[0][1] == bytes(st["notary"]["n_root"][0].cpu().numpy()), "notary chunk root vs CPU path"
        out["notary"] = {"one_core": round(1 / t1, 4), "all_core": round(nshard / tN, 4), "unit": "shards/s",
                         "kind": "reference",
                         "sample": f"1 / {nshard} shards of 8,192 txs: blob decode + Sender (reference crypto) + "
                                   "chunk root (restatement), one shard per thread"}
    if "pairing" in st:
        n1, nN = 64, max(2048, 64 * th)
        hin = st["pairing"]["pin"][:nN].cpu().numpy()
        pexp = st["pairing"]["pexp"][:nN].cpu().numpy()
        v = [None] * len(hin)
        t1 = _threads_run(lambda i: v.__setitem__(i, O.pairing_check(bytes(hin[i]))), list(range(n1)), 1)
        tN = _threads_run(lambda i: v.__setitem__(i, O.pairing_check(bytes(hin[i]))), list(range(len(hin))), th)
        assert [2 if x < 0 else x for x in v] == pexp[:len(v)].tolist(), "pairing oracle disagrees"
        out["pairing"] = {"one_core": round(n1 / t1, 1), "all_core": round(len(hin) / tN, 1), "unit": "checks/s",
                          "kind": "port", "sample": f"{n1} (1 thread) / {len(hin)} ({th} threads) 4-pair checks of the "
                                                    "configs[4] workload, oracle restatement of crypto/bn256/cloudflare"}
    return out


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 20 timed steps after 4 warm-up steps (r05: with 10 after 2 the headline leg read 114.7
    # instead of 117.3 M recoveries/s on the same box, profiles/r05/ab/ecrecover_steps.txt; the default
    # run still finishes in about a minute)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--legs", default=",".join(LEGS), help="comma list of " + ",".join(LEGS))
    ap.add_argument("--ecrecover-pipeline", type=int, default=2,
                    help="streams consecutive ecrecover (and collation-header) batches are spread over (2, the "
                         "default since r06: two batches in flight on dedicated-queue streams, as the other legs; "
                         "the roofline's kernel time then comes from a separate single-stream instrumented pass; "
                         "1: one stream, kernel time from HIP events over the timed region itself)")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="streams (shape instances) consecutive chunk-root (and Keccak, tx-root, POC) batches "
                         "are spread over")
    ap.add_argument("--pairing-pipeline", type=int, default=0,
                    help="streams (shape instances) consecutive pairing batches are spread over "
                         "(0 = auto: 6 below 65,536 checks per rank, else 1)")
    ap.add_argument("--pairing-checks", type=int, default=0,
                    help="checks per rank in the pairing leg (0 = configs[4]'s 65,536 split over the ranks; "
                         "8192 rehearses a rank of the 8-GPU run on one GPU)")
    ap.add_argument("--notary-pipeline", type=int, default=4,
                    help="streams (shape instances) consecutive notary partition steps are spread over "
                         "(r05, queues of their own: 1 / 2 / 3 deep 10,560 / 11,457 / 11,623 shards/s, "
                         "profiles/r05/ab/chunk_notary_depth.txt; r06: 4 since the N = 8 share of 13 shards "
                         "reads 1.125 ms per step four deep against 1.16-1.20 three deep, 100 shards equal at "
                         "2-4, profiles/r06/ab/notary_share_depths.txt)")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo rank plumbing only (no GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    legs = [x for x in args.legs.split(",") if x]
    bad = [x for x in legs if x not in LEGS]
    if bad:
        ap.error(f"unknown legs {bad}")

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}")

    ws, rank, local = dist_setup(args.dry_run)
    if args.dry_run:
        dry_run(args, ws, rank)
        if ws > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    import torch
    import gsv
    ctx = gsv.Context(local)
    stream = torch.cuda.Stream()
    dev = torch.device("cuda", local)
    res, state = {}, {}
    if "ecrecover" in legs:
        res["ecrecover"], state["ecrecover"] = leg_ecrecover(ctx, stream, dev, ws, rank, args)
    if "chunk_root" in legs:
        res["chunk_root"], state["chunk_root"] = leg_chunk_root(ctx, stream, dev, ws, rank, args)
    if "notary" in legs:
        res["notary"], state["notary"] = leg_notary(ctx, stream, dev, ws, rank, args)
    extras = {}
    if "keccak" in legs:
        extras["keccak256"] = leg_keccak(ctx, stream, dev, ws, rank, args)
    if "tx_root" in legs:
        extras["tx_root"] = leg_tx_root(ctx, stream, dev, ws, rank, args)
    if "poc" in legs:
        extras["proof_of_custody"] = leg_poc(ctx, stream, dev, ws, rank, args)
    if "headers" in legs and "ecrecover" in state:
        extras["collation_headers"] = leg_headers(ctx, stream, dev, ws, rank, args, state["ecrecover"]["sig"])
    if "pairing" in legs:
        res["pairing"], state["pairing"] = leg_pairing(ctx, stream, dev, ws, rank, args)

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        info = host_info()
        legs_cpu = cpu_baselines(ctx, legs, state, res, info)
        ec = legs_cpu.get("ecrecover")
        cpu = {"value": ec["all_core"] if ec else None, "unit": "sigs/s", "cores": info["threads_all_core"],
               "threads": info["threads_all_core"],
               "threads_basis": "one host thread per CPU of one GPU's share of an 8-GPU node (nproc / 8)",
               "cgroup_cpu_quota": info["cgroup_cpu_quota"], "affinity_cpus": info["affinity"],
               # the CPU time the threads can actually get: min(threads, the box's cgroup quota)
               "effective_cores": min(info["threads_all_core"], info["cgroup_cpu_quota"] or info["threads_all_core"]),
               "kind": ec["kind"] if ec else None, "sample": ec["sample"] if ec else None,
               "nproc": info["nproc"], "cpu_model": info["cpu_model"],
               "one_core": ec["one_core"] if ec else None, "all_core": ec["all_core"] if ec else None,
               "legs": legs_cpu}

    if rank == 0:
        ec = res.get("ecrecover")
        line = {
            "metric": "ecrecover sigs/sec + Keccak collation GB/s",
            "value": round(ec["rate"], 1) if ec else None,
            "unit": "sigs/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ec["dt"] / args.steps * 1e3, 3) if ec else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (GPU-signed secp256k1 signatures, keccak-derived keys/msgs/nonces)",
            "config": {"workload": "1M-signature secp256k1 ecrecover + Keccak-256 address derivation "
                                   "per GPU (BASELINE.json configs[1])",
                       "signatures_per_gpu": N_SIGS, "parallelism": f"shard-partitioned x{ws}",
                       "batches_in_flight": max(1, args.ecrecover_pipeline)},
            "roofline": ec["roofline"] if ec else None,
            "cpu_baseline": cpu,
        }
        if "chunk_root" in res:
            line["collation_GBps"] = res["chunk_root"]["collation_GBps"]
            line["chunk_root"] = res["chunk_root"]
        if "pairing" in res:
            line["bn256_pairing"] = res["pairing"]
        if "notary" in res:
            line["notary"] = res["notary"]
        if extras:
            line["collation_extras"] = extras
        print(json.dumps(line), flush=True)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
