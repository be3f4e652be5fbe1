#!/bin/bash
# Same-box A/B: the session-start library (lib_prev, 8f39c0c) against HEAD's (lib), alternating, K = 4 and 1.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/lib_ab.sh "" lib_prev lib lib_prev lib
