#!/bin/bash
# GPU-box script: GRBM_GUI_ACTIVE (cycles, summed over XCDs) per kernel for
# bench.py runs with the given extra args, to read the clock under load.
#   bash tools/run_clock.sh "--halfsize 1" "--halfsize 0"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d gpurun_out/clk$i -o run -- \
      python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $a > gpurun_out/clk$i.json 2> gpurun_out/clk$i.err || { tail -5 gpurun_out/clk$i.err; exit 1; }
  python3 - "$i" "$a" <<'PY'
import csv, glob, sys, collections
i, a = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/clk{i}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
        k = r["Kernel_Name"].split("(")[0]
        dur = (int(r.get("End_Timestamp", 0) or 0) - int(r.get("Start_Timestamp", 0) or 0))
        acc[k].append((float(r["Counter_Value"]), dur))
for k in ("k_verify_prep", "k_verify_dsm"):
    v = acc.get(k, [])
    if v:
        cyc = sum(x for x, _ in v) / len(v) / 8
        dur = sum(d for _, d in v) / len(v)
        print(a, k, "cycles/XCD", round(cyc), "dur_ns", dur, "GHz", round(cyc / dur, 3) if dur else None)
PY
done
