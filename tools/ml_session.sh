R=${GRAFT_REPO_ROOT:-$(pwd)}; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG:-r04d}_ml" -o run -- python3 "$R/tools/onnx_layers.py" run modnet:8:bf16 "$R/gpurun_out/${TAG:-r04d}_ml/launches.json" > "$R/gpurun_out/${TAG:-r04d}_ml.log" 2>&1 || exit $?
cd "$R"; python3 tools/onnx_layers.py report gpurun_out/${TAG:-r04d}_ml/launches.json gpurun_out/${TAG:-r04d}_ml/run_kernel_trace.csv 2>&1 | head -80
