cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_list.txt 2>&1 || true
PASSES="sq lds sq2" LABEL=salu bash tools/profile.sh
