bash tools/gpu_ab2.sh gpurun_out/rx "tests/test_gpu_engine.py tests/test_gpu_sizes.py tests/test_gpu_points.py" "abl/lib_base.so abl/lib_rx.so --rounds 6 --precision f64" && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_base.so abl/lib_rx.so --rounds 6 --precision f32 > gpurun_out/rx/ab32.json 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py abl/lib_base.so abl/lib_rx.so --rounds 4 --precision f64 --iters 0,1,2,3,4 > gpurun_out/rx/ab64_cnc4.json 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/rx/pmc_write32 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --precision f32 > gpurun_out/rx/pmc.log 2>&1
