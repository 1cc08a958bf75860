mkdir -p gpurun_out/r03a
python -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))" > gpurun_out/r03a/host.txt
cat /sys/fs/cgroup/cpu.max >> gpurun_out/r03a/host.txt 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 160 --timeout-method thread > gpurun_out/r03a/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r03a/bench.log 2>&1 || { echo "bench failed"; exit 1; }
bash tools/pmc_probe.sh ecrecover r03_ecr "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM" > gpurun_out/r03a/probe.log 2>&1 || { echo "probe failed"; exit 1; }
echo all done
