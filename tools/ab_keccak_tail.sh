#!/bin/bash
# (Record of the r06 run: the GSV_KECCAK_TAIL_X4 / GSV_KECCAK_WPE switches the variants were built with were removed after it; profiles/r06/ab/keccak_tail_loader.txt.)
# A/B of k_keccak256's final-block loader (run through gpurun from the repo root):
#   base   = in-tree at the time (whole 16-byte groups, five waves per SIMD forced; r06 run)
#   kx4w4  = whole 16-byte groups at the compiler's register count (106: four waves per SIMD)
#   kold   = one branch and one dword load per dword (r05/r06 form, 94 registers)
# Keccak tests on the in-tree library, then keccak_scale (400 k / 1.6 M messages) and the bench's keccak
# leg for each, twice in alternation, then one TA/SQ counter pass per library.
set -o pipefail
O=gpurun_out/kt; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_keccak.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in base kx4w4 kold; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L timeout -k 10 120 python tools/keccak_scale.py 400000 1600000 > $O/scale_${v}_$r.txt 2>&1 || { echo "$v scale failed"; tail -5 $O/scale_${v}_$r.txt; exit 1; }
    sed "s/^/$v /" $O/scale_${v}_$r.txt
    GSV_LIB_PATH=$L timeout -k 10 200 python bench.py --legs keccak --no-cpu-baseline --steps 20 > $O/bench_${v}_$r.log 2>&1 || { echo "$v bench failed"; exit 1; }
    tail -1 $O/bench_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['collation_extras']['keccak256']; print('$v leg', d['hashes_per_s'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base kold; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES -f csv -d $O/pmc_$v -o run -- python3 tools/keccak_scale.py 400000 > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/pmc_$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for v in ("base", "kold"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/kt/pmc_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_keccak256" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in sorted(agg.items())}, "dispatch rows", {k: len(x) for k, x in agg.items()})
PY
