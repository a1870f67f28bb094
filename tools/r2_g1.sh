set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
export PYTHONUNBUFFERED=1
for km in 4096:4096 4096:12288 4096:22016 11008:4096; do
  K=${km%%:*} M=${km##*:} timeout -k 10 120 python tools/gemv_stamps.py > gpurun_out/r2/stamps_$K_$M.log 2>&1 || exit $?
  echo "== K=${km%%:*} M=${km##*:}"; cat gpurun_out/r2/stamps_$K_$M.log
done
timeout -k 10 200 python tools/shape_sweep.py 4096:4096 4096:12288 4096:22016 11008:4096 > gpurun_out/r2/shapes_base.log 2>&1
cat gpurun_out/r2/shapes_base.log
