cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_spec_counts.py tests/test_gpu_baseline_shapes.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5_pre_t.log 2>&1 || exit 2
bash tools/ab_libs.sh 3 "--config 4 --steps 10 --warmup 3 --cpu-seconds 0 --no-host-inclusive" oncrpc4j_amd/libxdrgpu.so exp/lib_prev.so > gpurun_out/r5_pre_ab.jsonl 2> gpurun_out/r5_pre_ab.err || exit 3
