set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload e2e --steps 5 --warmup 1 --cpu-seconds 15 > gpurun_out/bench_e2e.log 2>&1 && echo E2E_OK && tail -1 gpurun_out/bench_e2e.log &&
timeout -k 10 400 python -u bench.py --workload e2e --steps 5 --warmup 1 --no-cpu-baseline --serial-extract > gpurun_out/bench_e2e_serial.log 2>&1 && echo E2E_SERIAL_OK && tail -1 gpurun_out/bench_e2e_serial.log | cut -c1-400
