# A/B of the pairing leg: base library and any variants/<name>/libgsv.so given as arguments
set -o pipefail
A="--steps 2 --warmup 1 --no-cpu-baseline --no-chunk-leg --no-notary-leg --no-extra-legs"
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -k 10 200 python -u bench.py $A > gpurun_out/ab_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['bn256_pairing']; print('$v', p['checks_per_s'], p['prepare_kernel_ms'], p['miller_kernel_ms'], p['final_exp_kernel_ms'])"
done
