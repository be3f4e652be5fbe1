cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bs8 -o run -- python3 $R/tools/band_sim.py 8 0 > $R/gpurun_out/bs8.log 2>&1
