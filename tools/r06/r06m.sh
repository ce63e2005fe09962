#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd $R
for rep in 1 2; do
  bash tools/ab_run.sh r06m "--config c3 --obs packed" c3p_base c3p_nt || exit 1
done
