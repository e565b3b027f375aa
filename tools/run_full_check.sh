set -o pipefail
OUT=${OUT:-r02q}
mkdir -p gpurun_out/${OUT:-r02q}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${OUT:-r02q}/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/${OUT:-r02q}/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/${OUT:-r02q}/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${OUT:-r02q}/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/${OUT:-r02q}/smoke.log; exit 1; }
tail -1 gpurun_out/${OUT:-r02q}/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${OUT:-r02q}/bench.json 2> gpurun_out/${OUT:-r02q}/bench.err || { echo bench failed; tail -20 gpurun_out/${OUT:-r02q}/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${OUT:-r02q}/bench.json')); print(d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
