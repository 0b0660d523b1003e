# bench.py A/B of library variants built by tools/ab_libs.sh (VARIANTS=...), alternating;
# one line per run into gpurun_out/abv.log: name value ms_per_step [policy-free, policy] update ms.
# AB_LIBS="name=path[:VAR=v,...] ..." (default: work and work-pf3), AB_ROUNDS (default 4).
mkdir -p gpurun_out; rm -f gpurun_out/abv.log
one() {  # name lib[:VAR=v,...]
  local lib=${2%%:*} sets=""; [ "$lib" != "$2" ] && sets=$(echo "${2#*:}" | tr , " ")
  env $sets MSACL_HIP_LIB_AB=1 MSACL_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/abv_b.out 2>gpurun_out/abv_b.err || return 1
  tail -1 gpurun_out/abv_b.out | python -c "import json,sys;d=json.load(sys.stdin);print('$1', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms_policy_free_policy'])" >> gpurun_out/abv.log
}
LIBS=${AB_LIBS:-"base=exp_libs/work/libmsacl_hip.so pf3=exp_libs/work-pf3/libmsacl_hip.so"}
for i in $(seq 1 ${AB_ROUNDS:-4}); do
  for v in $LIBS; do one ${v%%=*} ${v#*=} || exit 1; done
done
