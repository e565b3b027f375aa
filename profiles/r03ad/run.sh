#!/bin/bash
# r03ad: HEAD after the work-pulling revert -- full GPU suite (incl. the mixed-size concurrent drop-in test), smoke, default bench, config sweep
set -o pipefail
O=gpurun_out/r03ad; mkdir -p $O
export FD_DROPIN_SUMMARY=$O/dropin_c_callers.json
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rP > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
grep -h "C callers\|concurrent drop-in" $O/pytest_gpu.txt | head -5
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-200 $O/bench_default.json
bash tools/run_bench_configs.sh r03ad_configs > $O/configs.txt 2>&1 || { tail -20 $O/configs.txt; exit 1; }
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03ad_configs/bench_*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], round(d["value"] / 1e6, 2), "M/s", d["config"].get("workload", "")[:60])
PY
