mkdir -p gpurun_out
timeout -k 5 60 ./tests/cpp/build/gather_double_check > gpurun_out/gd.log 2>&1; echo "rc=$?" >> gpurun_out/gd.log
