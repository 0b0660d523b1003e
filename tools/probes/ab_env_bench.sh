# bench.py A/B over environment settings, alternating; one line per run into gpurun_out/abe.log:
# name value ms_per_step [policy-free, policy] update ms. AB_ENVS="name=VAR=v,VAR2=w ..." (a name
# with no settings runs the defaults), AB_ROUNDS (default 3).
mkdir -p gpurun_out; rm -f gpurun_out/abe.log
for i in $(seq 1 ${AB_ROUNDS:-3}); do
  for v in $AB_ENVS; do
    name=${v%%=*}; sets=""; [ "$name" != "$v" ] && sets=$(echo "${v#*=}" | tr , " ")
    env $sets timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/abe_b.out 2>gpurun_out/abe_b.err || exit 1
    tail -1 gpurun_out/abe_b.out | python -c "import json,sys;d=json.load(sys.stdin);print('$name', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms_policy_free_policy'])" >> gpurun_out/abe.log || exit 1
  done
done
