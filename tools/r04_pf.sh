#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/pf_ab.jsonl
for v in ${VARIANTS:-build pf3 pf6 pf8 build}; do
  if [ $v = build ]; then L=""; else L="MSACL_HIP_LIB=exp_libs/mlp_fused-$v/libmsacl_hip.so"; fi
  env $L timeout -k 10 200 python tools/mlp3_bench.py --reps 50 > gpurun_out/pf_one.jsonl 2> gpurun_out/pf_one.err \
    || { tail -5 gpurun_out/pf_one.err; exit 1; }
  sed "s/^{/{\"lib\": \"$v\", /" gpurun_out/pf_one.jsonl >> gpurun_out/pf_ab.jsonl
done
python3 - <<'PY'
import json, collections
rows=[json.loads(l) for l in open("gpurun_out/pf_ab.jsonl")]
t=collections.defaultdict(dict)
for r in rows:
    k=(r["kernel"], r.get("M"), r.get("N3"), r.get("groups"), r.get("keep"))
    t[k].setdefault(r["lib"], []).append(r["us"])
for k,v in t.items(): print(k, {l: x for l,x in v.items()})
PY
