#!/bin/bash
# packed-kernel A/B + phase stamps in one call (tools/r03_packed_ab.sh, tools/r03_packed_diag.sh)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/r03_packed_ab.sh && bash tools/r03_packed_diag.sh
