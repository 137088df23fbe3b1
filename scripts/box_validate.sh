#!/bin/bash
# GPU-box validation run: build check, box-tier tests, bench (default + single process),
# BASELINE configs, CPU profile of one consumer. Every step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
lscpu > gpurun_out/lscpu.txt 2>&1
cat /sys/fs/cgroup/cpu.max > gpurun_out/cgroup_cpu_max.txt 2>&1
python -c "import bench; print(bench.available_cpus())" > gpurun_out/available_cpus.txt 2>&1
timeout -k 10 300 python __graft_entry__.py > gpurun_out/entry.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --procs-per-rank 1 > gpurun_out/bench_1proc.json 2> gpurun_out/bench_1proc.err &&
timeout -k 10 600 python -m beholder_amd bench all --out gpurun_out/baseline_configs.json > gpurun_out/baseline.log 2>&1 &&
timeout -k 10 300 python scripts/profile_consumer.py > gpurun_out/cprofile_consumer.txt 2>&1
# rocprofv3 kernel trace of the flagship bench: documents that the path dispatches no GPU kernels
if [ $? -eq 0 ] && [ "${SKIP_ROCPROF:-0}" != "1" ]; then
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      -d "$GRAFT_REPO_ROOT/gpurun_out/rocprof" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" \
      --steps 3 --warmup 1 --procs-per-rank 1 > "$GRAFT_REPO_ROOT/gpurun_out/rocprof_bench.log" 2>&1 )
  echo "rocprof rc=$?" >> gpurun_out/rocprof_bench.log
  (find gpurun_out/rocprof -type f 2>/dev/null || echo "no rocprof output files (no kernel dispatches)") \
    > gpurun_out/rocprof_files.txt
fi
true
