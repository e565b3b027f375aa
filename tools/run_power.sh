#!/bin/bash
# GPU-box script: sample board power and clocks (rocm-smi, read-only) while a
# long C2 bench runs, to check whether k_verify_dsm runs at the power cap.
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8000 --warmup 2 > gpurun_out/power_bench.json 2> gpurun_out/power_bench.err &
B=$!
sleep 12
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout 20 rocm-smi --showpower --showclocks --showtemp --showmaxpower > gpurun_out/power_$i.txt 2>&1
  sleep 2
done
wait $B
rc=$?
timeout 20 rocm-smi --showpower --showclocks > gpurun_out/power_idle.txt 2>&1
for i in 1 2 3 4 5 6 7 8 9 10; do grep -hE "Package Power \(W\)|sclk clock level|junction" gpurun_out/power_$i.txt | tr "\n" " "; echo; done
grep -hiE "power \(|sclk" gpurun_out/power_idle.txt | head -5
tail -c 400 gpurun_out/power_bench.json
exit $rc
