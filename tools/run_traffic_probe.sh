#!/bin/bash
# GPU-box script: what the A/R table traffic costs k_verify_dsm.  The default
# build against the FD_DSM_TRAFFIC_PROBE builds (same instructions, tables
# L2-resident, wrong verdicts): launch and sustained timings (two rounds), then
# one FETCH_SIZE+GRBM and one WRITE_SIZE rocprofv3 pass per build.
# Build first: python firedancer_amd/build.py probe1 FD_DSM_TRAFFIC_PROBE=1 (and probe2 =2)
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/traffic_probe; mkdir -p $O
L=$R/firedancer_amd
lib() { if [ $1 = default ]; then unset FD_ED25519_HIP_LIB; else export FD_ED25519_HIP_LIB=$L/libfd_ed25519_hip_$1.so; fi; }
for rep in 1 2; do
  for v in default probe1 probe2; do
    lib $v
    timeout -k 10 150 python3 tools/dsm_traffic_probe.py 8 5 > $O/${v}_$rep.json 2> $O/${v}_$rep.err \
        || { echo "$v rc=$?"; tail -5 $O/${v}_$rep.err; exit 1; }
    cat $O/${v}_$rep.json
  done
done
for v in default probe1 probe2; do
  lib $v
  for c in FETCH_SIZE WRITE_SIZE; do
    pm="$c"; [ $c = FETCH_SIZE ] && pm="FETCH_SIZE GRBM_GUI_ACTIVE"
    timeout -s KILL 150 rocprofv3 --pmc $pm --kernel-trace --output-format csv -d $O/pmc_${v}_$c -o run -- \
        python3 tools/dsm_traffic_probe.py 0.5 3 > $O/pmc_${v}_$c.out 2> $O/pmc_${v}_$c.err \
        || { echo "$v $c rc=$?"; tail -5 $O/pmc_${v}_$c.err; exit 1; }
  done
done
python3 - $O <<'PY'
import csv, glob, json, os, sys
o = sys.argv[1]
out = {}
for v in ("default", "probe1", "probe2"):
    val = {}
    for c, names in (("FETCH_SIZE", ("FETCH_SIZE", "GRBM_GUI_ACTIVE")), ("WRITE_SIZE", ("WRITE_SIZE",))):
        rows = [r for f in glob.glob(os.path.join(o, f"pmc_{v}_{c}", "**", "*counter_collection.csv"), recursive=True)
                for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("k_verify_dsm")]
        for nm in names:
            xs = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == nm]
            val[nm] = sum(xs) / max(len(xs), 1)
    runs = [json.load(open(os.path.join(o, f"{v}_{r}.json"))) for r in (1, 2)]
    out[v] = {"dsm_ms": [x["dsm_ms"] for x in runs], "sustained_ms": [x["sustained_ms"] for x in runs],
              "fetch_x2_GB": round(2 * val["FETCH_SIZE"] * 1024 / 1e9, 3),
              "write_GB": round(val["WRITE_SIZE"] * 1024 / 1e9, 3),
              "grbm_cycles_per_xcd": round(val["GRBM_GUI_ACTIVE"] / 8)}
print(json.dumps(out))
json.dump(out, open(os.path.join(o, "summary.json"), "w"), indent=1)
PY
