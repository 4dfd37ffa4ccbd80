# rocprofv3 PC sampling (beta, host trap) of k_fill on the C3 batch: where the
# kernel's cycles go by code offset (diagnostics)
O=gpurun_out/${1:-r5pcs}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ABLATE_C3=1 ABLATE_STEPS=5 timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 50 --output-format csv -d $O/pcs -o run -- python3 tools/ablate.py > $O/pcs.out 2> $O/pcs.err
echo "rc=$?"
ls -la $O/pcs | head
