set -o pipefail
mkdir -p gpurun_out/c4ab
for sh in 1 2 3 6 1; do
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 8 --warmup 2 --dsm-share $sh > gpurun_out/c4ab/share$sh.json 2> gpurun_out/c4ab/share$sh.err || { tail -5 gpurun_out/c4ab/share$sh.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4ab/share$sh.json')); print('share $sh', d['value'], d.get('pcie_inclusive',{}).get('value') if isinstance(d.get('pcie_inclusive'),dict) else '')"
done
