set -o pipefail
bash tools/r06/gpu_tests_tl.sh adam1 "tests -m gpu" dcql && ALGO=cql timeout -k 10 400 bash tools/profiling/gpu_timeline.sh && grep -E "adam|step:" gpurun_out/tl_cql.txt
