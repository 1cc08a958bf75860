#!/bin/bash
# (Record of the r06 run; the GSV_GEN_LANE_MODE_MIN switch was removed after it, the threshold stays 4,096.)
# A/B of the generic-node lane-mode threshold (chunk_root.hip GEN_LANE_MODE_MIN: heights with at least
# that many generic nodes over the batch hash one node per lane, below it one node per 32-lane group
# with the cooperative Keccak).  base = in-tree (4,096); variants/glm<T> = threshold T.
# The bench's tx-root, chunk-root and POC legs per library, twice in alternation.
set -o pipefail
O=gpurun_out/glm; mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in base glm65536 glm262144 glm1073741824; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L timeout -k 10 300 python3 bench.py --legs tx_root,chunk_root,poc --no-cpu-baseline > $O/bench_${v}_r$rep.log 2>&1 || { echo "$v bench failed"; tail -5 $O/bench_${v}_r$rep.log; exit 1; }
    tail -1 $O/bench_${v}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['collation_extras']; print('$v', 'tx_root', e['tx_root']['txs_per_s'], e['tx_root']['ms_per_step'], 'ms | chunk', d['chunk_root']['collation_GBps'], 'GB/s | poc', e['proof_of_custody']['bodies_per_s'])"
  done
done
