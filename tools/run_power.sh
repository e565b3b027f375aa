#!/bin/bash
# GPU-box script: sample board power and clocks (rocm-smi, read-only) while a
# long C2 bench runs (default 8000 steps, ~64 s), to check whether
# k_verify_dsm runs at the power cap and that the rate holds over a minute.
# Usage: bash tools/run_power.sh [tag] [steps]
O=gpurun_out/${1:-power}; S=${2:-8000}; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --steps $S --warmup 2 > $O/power_bench.json 2> $O/power_bench.err &
B=$!
sleep 15
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout 20 rocm-smi --showpower --showclocks --showtemp --showmaxpower > $O/power_$i.txt 2>&1
  sleep 3
done
wait $B
rc=$?
timeout 20 rocm-smi --showpower --showclocks > $O/power_idle.txt 2>&1
for i in 1 2 3 4 5 6 7 8 9 10; do grep -hE "Package Power \(W\)|sclk clock level|junction" $O/power_$i.txt | tr "\n" " "; echo; done
grep -hiE "power \(|sclk" $O/power_idle.txt | head -5
tail -c 400 $O/power_bench.json
exit $rc
