"""A/B timing of libgsv.so variants (tools/build_variant.sh) on one bench leg, on the GPU box:

    python tools/ab_variants.py <leg> <variant|main> [...]

Runs `bench.py --legs <leg> --no-cpu-baseline` once per variant in its own process
(GSV_LIB_PATH=variants/<name>/libgsv.so; "main" = the in-tree library) and prints the leg's
throughput and kernel time.  Every run keeps bench.py's full-size parity assertions.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pick(line, leg):
    if leg == "ecrecover":
        return line["value"], line["roofline"]["kernel_avg_ms"]
    if leg == "pairing":
        p = line["bn256_pairing"]
        return p["checks_per_s"], (p["prepare_kernel_ms"], p["miller_kernel_ms"], p["final_exp_kernel_ms"])
    if leg == "chunk_root":
        return line["collation_GBps"], line["chunk_root"]["bottom_kernel_avg_ms"]
    if leg == "notary":
        return line["notary"]["shards_per_s"], line["notary"]["tx_kernels_ms_per_step"]
    return None, None


def main():
    leg, variants = sys.argv[1], sys.argv[2:]
    extra = os.environ.get("AB_ARGS", "").split()
    for v in variants:
        env = dict(os.environ)
        if v != "main":
            env["GSV_LIB_PATH"] = os.path.join(ROOT, "variants", v, "libgsv.so")
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--legs", leg, "--no-cpu-baseline"] + extra,
                           env=env, capture_output=True, text=True, timeout=600)
        lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
        if p.returncode or not lines:
            print(f"{v:12s} FAILED rc={p.returncode}\n{p.stderr[-1500:]}", flush=True)
            sys.exit(1)
        val, k = pick(json.loads(lines[0]), leg)
        print(f"{v:12s} {leg}: {val}  kernel_ms: {k}", flush=True)


if __name__ == "__main__":
    main()
