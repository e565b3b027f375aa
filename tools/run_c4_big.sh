# GPU-box script: C4 frags-per-step x tiles sweep at and above the default
# batch (bench.py --txns / --tiles), resident and PCIe-inclusive legs.
# Usage: bash tools/run_c4_big.sh <tag> "<txns> <tiles>" ...
T=${1:-c4big}; shift
O=gpurun_out/$T; mkdir -p $O
for cfg in "$@"; do
  set -- $cfg
  timeout -k 10 500 python bench.py --config c4 --txns $1 --tiles $2 --steps 8 --warmup 2 --no-cpu-baseline > $O/t$1_$2.json 2> $O/t$1_$2.err || { tail -5 $O/t$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/t$1_$2.json')); p=d['pcie_inclusive']; print('$1 $2', round(d['value']/1e6,2), 'pcie', round(p['value']/1e6,2), 'host', d['batch_host_ms'], 'gpu', d['batch_gpu_ms'], 'dsm', d['roofline']['avg_launch_ms'], d['roofline']['units_per_launch'])"
done
