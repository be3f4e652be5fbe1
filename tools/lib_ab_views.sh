R="$GRAFT_REPO_ROOT"
for L in lib lib_exp/rr12 lib lib_exp/rr12; do
  PTSVGF_LIB_DIR="$R/path-tracing-svgf_amd/$L" timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline --no-1080p --no-extras --view surface > "$R/gpurun_out/ab_s.json" 2>/dev/null || exit $?
  PTSVGF_LIB_DIR="$R/path-tracing-svgf_amd/$L" timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline --no-1080p --no-extras --width 1920 --height 1080 --frames-in-flight 6 > "$R/gpurun_out/ab_h.json" 2>/dev/null || exit $?
  python3 -c "
import json; s=json.loads(open('$R/gpurun_out/ab_s.json').read()); h=json.loads(open('$R/gpurun_out/ab_h.json').read())
print('$L surface', s['value'], '1080p', h['value'])"
done
