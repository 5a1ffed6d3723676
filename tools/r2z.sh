#!/bin/bash
# round-2 final profiles: rocprof kernel trace + stats (fp32 and bf16 steps), step PMC traffic
cd $GRAFT_REPO_ROOT
bash tools/profile.sh r2z_f32 && bash tools/profile.sh r2z_bf16 --dtype bf16 && bash tools/pmc_step.sh r2z_pmc
