mkdir -p gpurun_out/c4big
for cfg in "1048576 6" "2097152 6" "2097152 8" "1048576 6"; do
  set -- $cfg
  timeout -k 10 500 python bench.py --config c4 --txns $1 --tiles $2 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/c4big/t$1_$2.json 2> gpurun_out/c4big/t$1_$2.err || { tail -5 gpurun_out/c4big/t$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4big/t$1_$2.json')); p=d['pcie_inclusive']; print('$1 $2', round(d['value']/1e6,2), 'pcie', round(p['value']/1e6,2), d['batch_host_ms'], d['batch_gpu_ms'])"
done
