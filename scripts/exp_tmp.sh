set -euo pipefail
L=hockey-env_amd/hockey_amd/_lib
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
tail -1 gpurun_out/pytest_gpu.log
for lib in libhockey_hip.so libhockey_hip_noslp.so; do
  HK_LIB=$L/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 --warmup 200 > gpurun_out/bench_$lib.log 2>&1
  echo "$lib $(grep -o '"value": [0-9.e+]*' gpurun_out/bench_$lib.log)"
done
