set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in ${MODELS:-n s}; do
  cd yolo-infer_amd
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d ../gpurun_out/tr_$m -o tr -- python -m yolomi.profile --model $m --replay --reps 20 > ../gpurun_out/tr_$m.log 2>&1
  cd ..
  f=$(find gpurun_out/tr_$m -name "*kernel_trace.csv" | head -1)
  (cd yolo-infer_amd && python -m yolomi.profile --model $m --trace ../$f) > gpurun_out/prof_${m}_trace.txt 2>&1
done
