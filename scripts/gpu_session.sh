#!/bin/bash
# One gpurun call built from named steps (each under its own time limit; the call stops at the
# first step that ends in a fault, abort or timeout):
#   bash scripts/gpu_session.sh TAG step [step ...]
# steps: tests | smoke | pyt:FILES(,) | modes:CFG,STEPS,ROUNDS,M1/M2 | bench[:CFG] | drv[:CFG] (the driver's 20-after-5 command) | ab[:CFGS] | benchvar[:CFGS] | write[:CFG] | fetch[:CFG] |
#        bandsx:CFG,K,"F1|F2" | sq[:CFG] | waits[:CFG] | xstamps:CFG[,K[,VARIANT[,RANK]]] | trace[:CFG] | strong[:CFG] | drvab[:CFG[,ROUNDS]] | py:<script args...> (quoted)
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -n ${TAILN:-6}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -eq 0 ] || [ -n "$KEEP_GOING" ] || exit $rc
}
libs() { echo base; ls build/variants/*.so 2>/dev/null; }
pmc() {  # pmc <name> <cfg> <counters...>
  local name=$1 cfg=$2; shift 2
  for lib in $(libs); do
    local ln=$(basename $lib .so)
    if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
    run ${name}_${ln}_$cfg 120 rocprofv3 --pmc "$@" -d "$OUT/${name}_${ln}_$cfg" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config "$cfg" --steps 5 --warmup 1 --cpu-seconds 0 --parts 1 --no-verify
  done
  unset VRT_LIB
}
for st in "$@"; do
  arg=${st#*:}; [ "$arg" = "$st" ] && arg=""
  case ${st%%:*} in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pyt) run pyt_$(echo $arg | tr -c 'a-zA-Z0-9' '_' | cut -c1-40) 600 python -u -m pytest ${arg//,/ } -x -v --timeout 200 --timeout-method thread ;;
    modes)  # bench A/B over vrt_set_exact_pass modes: modes:CFG,STEPS,ROUNDS,M1/M2/... (driver shape: STEPS 20)
      IFS=, read mc ms mr mm <<< "$arg"
      for ((i = 1; i <= ${mr:-2}; i++)); do
        for m in ${mm//\// }; do
          TAILN=0 run modes_${mc}_s${ms}_m${m}_$i 150 python bench.py --config $mc --steps ${ms:-20} --warmup 5 --cpu-seconds 0 --no-verify --exact-pass $m
          echo "modes $mc steps ${ms} ep$m $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/modes_${mc}_s${ms}_m${m}_$i.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $OUT/modes_${mc}_s${ms}_m${m}_$i.log | head -1) $(grep -o '"frame_latency_ms": [0-9.]*' $OUT/modes_${mc}_s${ms}_m${m}_$i.log | head -1)"
        done
      done ;;
    bench) run bench_${arg:-C3} 300 python bench.py --config ${arg:-C3} ;;
    drv) run drv_${arg:-C3} 300 python bench.py --config ${arg:-C3} --steps 20 --warmup 5 ;;
    ab) run ab 600 python -u scripts/ab.py --rounds 8 --configs ${arg:-C1,C2,C3,C4} ;;
    benchvar)
      for lib in $(libs); do
        ln=$(basename $lib .so)
        if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
        for cfg in ${arg//,/ }; do
          run bench_${ln}_$cfg 200 python bench.py --config $cfg --cpu-seconds 0 --no-verify
        done
      done; unset VRT_LIB ;;
    write) pmc write ${arg:-C3} WRITE_SIZE ;;
    fetch) pmc fetch ${arg:-C3} FETCH_SIZE ;;
    waits) pmc waits ${arg:-C3} SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM ;;
    sq) pmc sq ${arg:-C3} SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD ;;
    util) pmc util ${arg:-C3} SQ_WAVES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES ;;
    sca) pmc sca ${arg:-C3} SQ_WAVES SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_BRANCH ;;
    trace) run trace_${arg:-C3} 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_${arg:-C3}" -o run --output-format csv -- \
             python3 "$ROOT/bench.py" --config ${arg:-C3} --steps 20 --warmup 3 --cpu-seconds 0 ;;
    xstamps)  # exact-pass wave timeline (build/diag/libvrt_stamps.so: make variant NAME=stamps DEFS=-DVRT_STAMPS)
      IFS=, read xc xk xv xr <<< "$arg"
      VRT_LIB=$ROOT/build/diag/libvrt_stamps$xv.so run xstamps${xv}_${xc}_k${xk:-1}_r${xr:-0} 120 python -u scripts/exact_stamps.py --config $xc --ranks ${xk:-1} --rank ${xr:-0} ;;
    varmodes)  # every library (base + build/variants/*.so) x exact-pass modes: varmodes:CFG,STEPS,M1/M2
      IFS=, read vc vs vm <<< "$arg"
      for lib in $(libs); do
        ln=$(basename $lib .so)
        if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
        for m in ${vm//\// }; do
          TAILN=0 run vm_${ln}_${vc}_s${vs}_m$m 150 python bench.py --config $vc --steps ${vs:-20} --warmup 5 --cpu-seconds 0 --no-verify --exact-pass $m
          echo "varmodes $ln $vc steps $vs ep$m $(grep -o '"ms_per_step": [0-9.]*' $OUT/vm_${ln}_${vc}_s${vs}_m$m.log | head -1) $(grep -o '"frame_latency_ms": [0-9.]*' $OUT/vm_${ln}_${vc}_s${vs}_m$m.log | head -1)"
        done
      done; unset VRT_LIB ;;
    drvx)  # driver-shaped runs with extra bench flags, ROUNDS alternating: drvx:CFG,ROUNDS,"FLAGS1|FLAGS2|..."
      IFS=, read xc xr xf <<< "$arg"
      IFS='|' read -ra xfl <<< "$xf"
      for ((i = 1; i <= ${xr:-2}; i++)); do
        for j in "${!xfl[@]}"; do
          TAILN=0 run drvx_${xc}_${j}_$i 150 python bench.py --config $xc --steps 20 --warmup 5 --cpu-seconds 0 --no-verify --frame-events ${xfl[$j]}
          echo "drvx $xc [${xfl[$j]}] $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/drvx_${xc}_${j}_$i.log | head -1) $(grep -o '"frame_latency_ms": [0-9.]*' $OUT/drvx_${xc}_${j}_$i.log | head -1) $(grep -o '"frame_events_ms": \[[^]]*\]' $OUT/drvx_${xc}_${j}_$i.log | head -1)"
        done
      done ;;
    benchx)  # bench runs per flag set, ROUNDS alternating: benchx:CFG,STEPS,ROUNDS,"FLAGS1|FLAGS2"
      IFS=, read yc ys yr yf <<< "$arg"
      IFS='|' read -ra yfl <<< "$yf"
      for ((i = 1; i <= ${yr:-2}; i++)); do
        for j in "${!yfl[@]}"; do
          TAILN=0 run benchx_${yc}_s${ys}_${j}_$i 150 python bench.py --config $yc --steps $ys --warmup 5 --cpu-seconds 0 --no-verify ${yfl[$j]}
          echo "benchx $yc s$ys [${yfl[$j]}] $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/benchx_${yc}_s${ys}_${j}_$i.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $OUT/benchx_${yc}_s${ys}_${j}_$i.log | head -1) $(grep -o '"frame_latency_ms": [0-9.]*' $OUT/benchx_${yc}_s${ys}_${j}_$i.log | head -1)"
        done
      done ;;
    drvab)  # the driver's 20-frame command, ROUNDS alternating rounds over base + build/variants/*.so
      IFS=, read dc dr <<< "$arg"
      for ((i = 1; i <= ${dr:-4}; i++)); do
        for lib in $(libs); do
          ln=$(basename $lib .so)
          if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
          TAILN=0 run drvab_${ln}_${dc:-C3}_$i 120 python bench.py --config ${dc:-C3} --steps 20 --warmup 5 --cpu-seconds 0 --no-verify
          echo "drvab ${ln} ${dc:-C3} $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/drvab_${ln}_${dc:-C3}_$i.log | head -1) $(grep -o '"frame_latency_ms": [0-9.]*' $OUT/drvab_${ln}_${dc:-C3}_$i.log | head -1)"
        done
      done; unset VRT_LIB ;;
    benchab)  # steady-state bench (STEPS frames), ROUNDS alternating rounds over base + variants: benchab:CFG,STEPS,ROUNDS[,FLAGS]
      IFS=, read bc bs br bf <<< "$arg"
      for ((i = 1; i <= ${br:-2}; i++)); do
        for lib in $(libs); do
          ln=$(basename $lib .so)
          if [ $lib = base ]; then unset VRT_LIB; else export VRT_LIB=$ROOT/$lib; fi
          TAILN=0 run benchab_${ln}_${bc}_$i 150 python bench.py --config $bc --steps ${bs:-500} --warmup 20 --cpu-seconds 0 --no-verify $bf
          echo "benchab ${ln} ${bc} $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/benchab_${ln}_${bc}_$i.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $OUT/benchab_${ln}_${bc}_$i.log | head -1) $(grep -o '"frame_latency_ms": [0-9.]*' $OUT/benchab_${ln}_${bc}_$i.log | head -1)"
        done
      done; unset VRT_LIB ;;
    strongm)  # K-way split rehearsal of every rank over exact-pass modes: strongm:CFG,K,M1/M2
      IFS=, read sc sk sm <<< "$arg"
      for m in ${sm//\// }; do
        for ((r = 0; r < sk; r++)); do
          TAILN=0 run strongm_${sc}_k${sk}_r${r}_m$m 150 python bench.py --config $sc --rehearse-ranks $sk \
            --rehearse-rank $r --steps 400 --warmup 100 --cpu-seconds 0 --no-verify --exact-pass $m
          echo "strongm $sc k$sk r$r ep$m $(grep -o '"kernel_ms": [0-9.]*' $OUT/strongm_${sc}_k${sk}_r${r}_m$m.log | head -1)"
        done
      done ;;
    bandsx)  # every rank's band of a K-way split per flag set, slowest last: bandsx:CFG,K,"FLAGS1|FLAGS2"
      IFS=, read bc bk bf <<< "$arg"
      IFS='|' read -ra bfl <<< "$bf"
      for j in "${!bfl[@]}"; do
        worst=0
        for ((r = 0; r < bk; r++)); do
          TAILN=0 run bandsx_${bc}_k${bk}_${j}_r$r 150 python bench.py --config $bc --rehearse-ranks $bk --rehearse-rank $r \
            --steps 400 --warmup 100 --cpu-seconds 0 --no-verify ${bfl[$j]}
          km=$(grep -o '"kernel_ms": [0-9.]*' $OUT/bandsx_${bc}_k${bk}_${j}_r$r.log | head -1 | grep -o '[0-9.]*$')
          echo "bandsx $bc k$bk [${bfl[$j]}] r$r kernel_ms $km $(grep -o '"launches_in_flight": [0-9.]*' $OUT/bandsx_${bc}_k${bk}_${j}_r$r.log | head -1)"
          worst=$(python3 -c "print(max($worst, ${km:-0}))")
        done
        echo "bandsx $bc k$bk [${bfl[$j]}] slowest $worst"
      done ;;
    rep)  # one rank's band of a K-way split in N separate processes per flag set: rep:CFG,K,R,N,"FLAGS1|FLAGS2"
      IFS=, read rc rk rr rn rf <<< "$arg"
      IFS='|' read -ra rfl <<< "$rf"
      for ((i = 1; i <= ${rn:-3}; i++)); do
        for j in "${!rfl[@]}"; do
          TAILN=0 run rep_${rc}_k${rk}_r${rr}_${j}_$i 150 python bench.py --config $rc --rehearse-ranks $rk --rehearse-rank $rr \
            --steps 400 --warmup 100 --cpu-seconds 0 --no-verify ${rfl[$j]}
          echo "rep $rc k$rk r$rr [${rfl[$j]}] $i $(grep -o '"kernel_ms": [0-9.]*' $OUT/rep_${rc}_k${rk}_r${rr}_${j}_$i.log | head -1) $(grep -o '"launches_in_flight": [0-9.]*' $OUT/rep_${rc}_k${rk}_r${rr}_${j}_$i.log | head -1) $(grep -o '"frame_latency_ms": [0-9.]*' $OUT/rep_${rc}_k${rk}_r${rr}_${j}_$i.log | head -1)"
        done
      done ;;
    strong)  # strong-scaling rehearsal: every rank's band of the K-way split for K = 2, 4, 8
      for k in 2 4 8; do
        for ((r = 0; r < k; r++)); do
          TAILN=0 run strong_${arg:-C3}_k${k}_r$r 200 python bench.py --config ${arg:-C3} --rehearse-ranks $k \
            --rehearse-rank $r --steps 400 --warmup 100 --cpu-seconds 0 --no-verify
          echo "strong ${arg:-C3} k$k r$r $(grep -o '"kernel_ms": [0-9.]*' $OUT/strong_${arg:-C3}_k${k}_r$r.log | head -1)"
        done
      done ;;
    py) run py_$(echo $arg | tr -c 'a-zA-Z0-9' '_' | cut -c1-40) 600 python -u $arg ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
exit 0
