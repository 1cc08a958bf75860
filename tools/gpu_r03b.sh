bash tools/gpu_r03a.sh || exit 1
bash tools/ab_chunk_top.sh top4 > gpurun_out/abtop.log 2>&1 || { echo "abtop failed"; exit 1; }
echo combo done
