# fixed per-step costs: GPU suite, bench slices, slice timeline
O=gpurun_out/${1:-r5f}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python bench.py --no-cpu --no-c4 --no-c5 --no-extra --no-c4t --steps 100 > $O/slices.json 2> $O/slices.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/slice_trace.py 8 0 30 > $O/traced.txt 2>&1 || exit 1
