# band sim with SVGF-stream occupancy (8 bands, exchanges modelled), then the final rocprof passes
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/band_sim.py 8 > gpurun_out/band_sim_g24.log 2>&1 || exit $?
FIF=4 bash tools/gpu_profile.sh r03fk4 && FIF=4 VIEW=surface bash tools/gpu_profile.sh r03fk4s && \
FIF=1 PASSES=trace bash tools/gpu_profile.sh r03fk1 && FIF=1 VIEW=surface PASSES=trace bash tools/gpu_profile.sh r03fk1s
