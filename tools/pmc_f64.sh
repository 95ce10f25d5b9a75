#!/bin/bash
# PMC passes over an exact-f64 kernel (KRE, default trellis_fwd_f64; also backtrack_f64) in the config-4 bench (one
# 65,536-sequence launch per step): HBM traffic (FETCH_SIZE, WRITE_SIZE: one pass each, the
# gfx950 FETCH_SIZE x2 correction in tools/pmc_summary.py) and SQ issue/wait counters + the
# clock (GRBM_GUI_ACTIVE).  One --pmc group per run, kernel trace only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pmc_f64}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-f32-extra --no-configs ${PMC_ARGS:-}"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${T_PMC:-240} rocprofv3 --pmc $C --kernel-include-regex "${KRE:-trellis_fwd_f64}" -d $OUT/$C -o p \
    --output-format csv -- python3 $R/bench.py $ARGS > $OUT/$C.log 2>&1 || exit $?
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json | head -8
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS" \
         "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -k 10 ${T_PMC:-240} rocprofv3 --pmc $G --kernel-include-regex "${KRE:-trellis_fwd_f64}" -d $OUT/g$i -o p \
    --output-format csv -- python3 $R/bench.py $ARGS > $OUT/g$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY' > $OUT/sq_summary.txt
import csv, glob, os, sys, collections
out = sys.argv[1]
rows = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "g*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        rows[row["Counter_Name"]].append((int(row.get("Dispatch_Id", 0)), float(row["Counter_Value"]),
                                          float(row.get("End_Timestamp", 0)) - float(row.get("Start_Timestamp", 0))))
tot = {}
dur = {}
for k, v in rows.items():
    v.sort()
    keep = v[len(v) // 2:]  # warmup launch + timed launch: keep the timed one
    tot[k] = sum(x[1] for x in keep)
    dur[k] = sum(x[2] for x in keep)
for k in sorted(tot):
    print(f"{k:30s} {tot[k]:.4e}")
w = tot.get("SQ_WAVE_CYCLES", 0)
if w:
    for k in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
              "SQ_ACTIVE_INST_ANY"):
        if k in tot:
            print(f"{k} / SQ_WAVE_CYCLES = {tot[k] / w:.3f}")
if tot.get("GRBM_GUI_ACTIVE") and dur.get("GRBM_GUI_ACTIVE"):
    # MI355X_MICROARCH.md DVFS note: GRBM_GUI_ACTIVE sums the 8 XCDs
    print(f"effective clock = {tot['GRBM_GUI_ACTIVE'] / 8 / (dur['GRBM_GUI_ACTIVE'] * 1e-9) / 1e9:.3f} GHz "
          f"(kernel {dur['GRBM_GUI_ACTIVE'] * 1e-6:.2f} ms)")
PY
cat $OUT/sq_summary.txt
# traffic + the effective clock in one summary (what bench.py reads from profiles/)
python3 - "$OUT" "${TAG:-pmc_f64}" <<'PY'
import json, re, sys, os
out, tag = sys.argv[1], sys.argv[2]
d = json.load(open(os.path.join(out, "traffic.json")))
m = re.search(r"effective clock = ([0-9.]+) GHz \(kernel ([0-9.]+) ms\)", open(os.path.join(out, "sq_summary.txt")).read())
if m:
    d["clock_ghz"] = float(m.group(1))
    d["kernel_ms_pmc"] = float(m.group(2))
d["source"] = f"rocprofv3 --pmc passes, gpurun_out/{tag}"
json.dump(d, open(os.path.join(out, "pmc_merged.json"), "w"), indent=1)
print(json.dumps(d)[:300])
PY
