set -o pipefail
for a in 0 1 3 7; do
  DGMC_SC_FZ_ABL=$a bash tools/prof_quick.sh abl$a > /dev/null 2>&1 || exit $?
  echo "abl=$a: $(grep 'slot_conv_ws_kernel<true' gpurun_out/abl$a/step.txt | cut -c1-40)"
done
echo "fused off: "; DGMC_AMD_FUSED_RELU_BWD=0 bash tools/prof_quick.sh ablx > /dev/null 2>&1; grep 'slot_conv_ws_kernel<true\|colsum\|step span' gpurun_out/ablx/step.txt | cut -c1-60
