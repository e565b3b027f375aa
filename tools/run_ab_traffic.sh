#!/bin/bash
# GPU-box script: k_verify_dsm HBM-side bytes per launch (FETCH_SIZE x2 +
# WRITE_SIZE, one rocprofv3 --pmc pass each, no trace domains) for build
# variants.  Usage: bash tools/run_ab_traffic.sh <tag> <variant>...  ("" = default)
export TMPDIR=/tmp
R=$(pwd); T=$1; shift; O=$R/gpurun_out/abt_$T; mkdir -p $O
for v in "$@"; do
  if [ -n "$v" ]; then export FD_ED25519_HIP_LIB=$v; else unset FD_ED25519_HIP_LIB; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${v:-default}_$c -o run -- \
        python3 bench.py --contexts 1 --no-cpu-baseline --steps 2 --warmup 1 > $O/${v:-default}_$c.out 2> $O/${v:-default}_$c.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v $c rc=$rc"; tail -5 $O/${v:-default}_$c.err; exit $rc; }
  done
  python3 - $O ${v:-default} <<'PY'
import csv, glob, sys, os
o, v = sys.argv[1], sys.argv[2]
val = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    xs = [float(r["Counter_Value"]) for f in glob.glob(os.path.join(o, f"{v}_{c}", "**", "*counter_collection.csv"), recursive=True)
          for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("k_verify_dsm")]
    val[c] = sum(xs) / len(xs) * 1024   # KB -> bytes
print(v, "dsm GB/launch: fetch x2", round(2 * val["FETCH_SIZE"] / 1e9, 3), "write", round(val["WRITE_SIZE"] / 1e9, 3),
      "total", round((2 * val["FETCH_SIZE"] + val["WRITE_SIZE"]) / 1e9, 3))
PY
done
