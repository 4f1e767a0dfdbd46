cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/r03_s31; mkdir -p $OUT
b() { local name=$1; shift
  timeout -k 10 200 python bench.py --cpu-seconds 0 --no-verify "$@" > $OUT/$name.log 2>&1 || exit $?
  python -c "import json,sys;l=[x for x in open('$OUT/$name.log') if x.startswith('{')][-1];d=json.loads(l);print('$name', d['ms_per_step'], d.get('kernel_ms'))"; }
b drv --steps 20 --warmup 5
b drv_dw1000 --steps 20 --warmup 5 --device-warmup-ms 1000
b drv_w100 --steps 20 --warmup 100
b s100 --steps 100 --warmup 5
b s1000 --steps 1000 --warmup 5
b drv_l1 --steps 20 --warmup 5 --lanes 1
b drv_l2 --steps 20 --warmup 5 --lanes 2
b drv_x0 --steps 20 --warmup 5 --exact-pass 0
b drv_x2 --steps 20 --warmup 5 --exact-pass 2
b k2_x0 --rehearse-ranks 2 --steps 500 --warmup 200 --exact-pass 0
b k2_x1 --rehearse-ranks 2 --steps 500 --warmup 200 --exact-pass 1
b k4_x2 --rehearse-ranks 4 --steps 500 --warmup 200 --exact-pass 2
b k8_x2 --rehearse-ranks 8 --steps 500 --warmup 200 --exact-pass 2
b c4k8_x2 --config C4 --rehearse-ranks 8 --steps 500 --warmup 200 --exact-pass 2
b c4k2_x0 --config C4 --rehearse-ranks 2 --steps 500 --warmup 200 --exact-pass 0
