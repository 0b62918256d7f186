#!/bin/bash
# dev: PMC counters of the vocoder convs (separate passes; FETCH_SIZE alone)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
P="$R/gpurun_out/pmc_voc"
rm -rf "$P"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/a" -o a -- python3 "$R/tools/dev/voc_only.py" 128 > "$R/gpurun_out/pmc_voc_a.log" 2>&1 || { echo "pmc a failed"; tail -5 "$R/gpurun_out/pmc_voc_a.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA --output-format csv -d "$P/b" -o b -- python3 "$R/tools/dev/voc_only.py" 128 > "$R/gpurun_out/pmc_voc_b.log" 2>&1 || { echo "pmc b failed"; tail -5 "$R/gpurun_out/pmc_voc_b.log"; exit 1; }
python3 - "$P" <<'PY'
import csv, glob, sys, collections
P = sys.argv[1]
for sub in ("a", "b"):
    f = glob.glob(f"{P}/{sub}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"][:40] + " g" + row.get("Grid_Size", row.get("Grid_Size_X", ""))
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        cnt[(k, row["Counter_Name"])] += 1
    for k, d in sorted(agg.items(), key=lambda kv: -max(kv[1].values()))[:8]:
        print(sub, k, {c: f"{v / cnt[(k, c)]:.3g}" for c, v in d.items()})
PY
