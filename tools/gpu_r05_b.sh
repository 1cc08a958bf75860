#!/bin/bash
# r05 call B: every GPU test on the current tree; VALU issue costs of the Keccak bit ops (occupancy
# microbenchmark); the N = 8 rank batch of configs[4] under forced Miller splits at depth 3 / 4; leg-only
# PMC passes of the chunk root and Keccak legs (achieved waves per SIMD)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05b; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/microbench_occ.hip -o /tmp/mbocc && $T 300 /tmp/mbocc > $O/microbench_occ_ops.txt 2>&1 || { echo microbench failed; tail $O/microbench_occ_ops.txt; exit 1; }
cat $O/microbench_occ_ops.txt
for k in 1 2 4; do
  GSV_BN_PAIRS_PER_LANE=$k SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE="3,4" $T 240 python -u tools/pairing_sweep.py 8192 > $O/sweep8192_k$k.txt 2>&1 || { echo sweep $k failed; tail $O/sweep8192_k$k.txt; exit 1; }
  grep checks $O/sweep8192_k$k.txt | sed "s/^/k=$k /"
done
bash tools/profile_round.sh r05b chunk_root keccak > $O/profile.log 2>&1 || { echo profile failed; tail $O/profile.log; exit 1; }
cp gpurun_out/prof/r05b/pmc_*.json gpurun_out/prof/r05b/kernel_stats_*.csv $O/
find gpurun_out/prof/r05b -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
python3 -c "
import json
for g in ('chunk_root','keccak'):
    d=json.load(open('$O/pmc_%s.json'%g))
    for k,v in d.items():
        if 'level' in k or 'keccak256' in k or 'top' in k: print(g, k, {x: v.get(x) for x in ('avg_ms','mean_waves_per_simd','valu_issue_per_simd_cycle','vgpr','profiled_clock_ghz','wait_inst_any_frac','wait_any_frac')})
"
