set -o pipefail
# (Record of the r06 run: the GSV_NOTARY_FAKE_SIGHASH switch the variant was built with, -DGSV_NOTARY_FAKE_SIGHASH making PreStream::at return (k * 7 + seg_lo) without reading memory, was removed after it; profiles/r06/ab/notary_fake_sighash.txt.)
O=gpurun_out/nf; mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in base nfake; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L GSV_MAX_SIDE_STREAMS=0 NOTARY_DEPTHS=1 NOTARY_STEPS=12 timeout -k 10 300 python3 tools/notary_sweep.py 128 100 > $O/${v}_r$rep.txt 2>&1 || { echo "$v sweep failed"; tail $O/${v}_r$rep.txt; exit 1; }
    grep shards $O/${v}_r$rep.txt | sed "s/^/$v /"
  done
done
