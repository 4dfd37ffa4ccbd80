# k_rows on one block per CU: GPU suite, slices, kernel-trace summary
O=gpurun_out/${1:-r5r}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python bench.py --no-cpu --no-c4 --no-c5 --no-extra --no-c4t --steps 100 > $O/slices.json 2> $O/slices.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-side --no-steady > $O/trace_bench.json 2> $O/trace.err || exit 1
