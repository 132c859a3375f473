set -o pipefail
for pr in 0 1 2 3; do
  D3A_SMALL_PROBE=$pr ALGO=bcq timeout -k 10 300 bash tools/profiling/gpu_timeline.sh || exit 1
  echo "probe $pr"; grep -E "mlp_small_kernel<2, ., true>|step:" gpurun_out/tl_bcq.txt
done
