#!/bin/bash
# GPU-box script: instruction-cache counters (one rocprofv3 PMC pass, SQ block
# only) over bench.py --contexts 1: are the engine kernels' instruction
# fetches served by the CU instruction cache?
# Usage: bash tools/run_icache_pmc.sh <tag> [bench args...]
export TMPDIR=/tmp
T=${1:-icache}; shift
O=$PWD/gpurun_out/$T; mkdir -p $O
G="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/p -o run -- \
    python3 bench.py --contexts 1 --no-cpu-baseline --steps 2 --warmup 1 "$@" > $O/out.json 2> $O/err.txt
rc=$?; echo "icache pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/err.txt; exit $rc; }
python3 - $O <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in ("k_verify_prep", "k_verify_dsm"):
    m = {c: sum(v) / len(v) for c, v in acc[k].items()}
    print(k, {c: round(v) for c, v in sorted(m.items())})
    if m.get("SQC_ICACHE_REQ"):
        print("  hit rate", round(m["SQC_ICACHE_HITS"] / m["SQC_ICACHE_REQ"], 4),
              "ifetch latency (cycles)", round(m.get("SQ_IFETCH_LEVEL", 0) / max(m.get("SQ_IFETCH", 1), 1), 1))
PY
