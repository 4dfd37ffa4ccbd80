O=gpurun_out/${1:-r5sl}; mkdir -p $O
timeout -k 10 300 python tools/slice_trace.py 8 0 30 > $O/plain.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/slice_trace.py 8 0 30 > $O/traced.txt 2>&1 || exit 1
