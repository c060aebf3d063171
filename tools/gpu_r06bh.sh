#!/bin/bash
# r06bh: closing evidence at the final HEAD (after the ROIAlign branch test hook) -- every GPU test, smoke, the default bench line (with the nested config-3 record), and
# the rocprofv3 kernel trace + stats of the config-2 bench (its conv average vs the line's hipEvents)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06bh_gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r06bh_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06bh_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06bh_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06bh_smoke.log; exit 1; }
tail -1 gpurun_out/r06bh_smoke.log
timeout -k 10 560 python -u bench.py > gpurun_out/r06bh_bench.json 2> gpurun_out/r06bh_bench.err || { echo "bench failed"; tail -20 gpurun_out/r06bh_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06bh_bench.json'));e=d['e2e'];print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'],e.get('value'),e.get('child_wall_s'),e['gate_detector']['traffic_per_call'],e['roofline']['traffic'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r06bh_trace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-throughput-mode --no-e2e > "$R/gpurun_out/prof_r06bh_trace.log" 2>&1 && echo trace ok
