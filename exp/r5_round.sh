O=gpurun_out/${1:?tag}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -5 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
