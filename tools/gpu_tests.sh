O=gpurun_out/${1:-gpu_tests}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
echo "rc=$?" >> $O/pytest_gpu.txt
