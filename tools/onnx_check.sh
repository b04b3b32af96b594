timeout -k 10 300 python -u -m pytest tests/test_gpu_onnx.py tests/test_gpu_face.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r04n_onnx_tests.log 2>&1; tail -1 gpurun_out/r04n_onnx_tests.log
timeout -k 10 300 python tools/bench_onnx.py --only-modnet --batch 8 --iters 50 > gpurun_out/r04n_b8.log 2>&1 && grep -h '^{' gpurun_out/r04n_b8.log | cut -c1-130
