#!/usr/bin/env bash
# Round 3 PMC traffic passes: C3 GROUP BY (4 quads per thread now) and the
# many-key partitioned GROUP BY (1e9 rows x 1e6 keys).  Each counter in its
# own rocprofv3 pass (tools/pmc_run.sh).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/pmc_run.sh group 1e9 > /dev/null
bash tools/pmc_run.sh group 1e9 "--keys 1000000" group_wide > /dev/null
echo done
