#!/bin/bash
# A/B: leaf chunk of 2 (SLP off leaves registers for it), resident-wave estimates 24 / 28 per CU, against HEAD.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/lib_ab.sh "" lib lib_exp/chunk2 lib_exp/rw24 lib_exp/rw28 lib lib_exp/chunk2 lib_exp/rw24 lib_exp/rw28
