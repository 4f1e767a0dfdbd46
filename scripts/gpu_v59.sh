# v59: wave timeline with the certified/exact split, then per-wave exact steps beside it
cd $GRAFT_REPO_ROOT
bash scripts/gpu_stamps.sh v60stamps C3 || exit $?
timeout -k 10 200 python scripts/wave_steps.py --config C3 --stamps gpurun_out/v60stamps/stamps_C3.npz > gpurun_out/v60stamps/wave_steps.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/v60stamps/wave_steps.log | tail -28; exit $rc
