# bench.py (default C3) for the default library and each build/variants/*.so
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O; shift
for lib in base build/variants/*.so; do
  name=$(basename $lib .so)
  if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$GRAFT_REPO_ROOT/$lib; fi
  for cfg in "$@"; do
    timeout -k 10 200 python bench.py --config $cfg --cpu-seconds 0 > $O/bench_${name}_$cfg.log 2>&1 || exit 1
    echo "$name $cfg $(tail -1 $O/bench_${name}_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
