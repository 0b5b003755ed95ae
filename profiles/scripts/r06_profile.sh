#!/bin/bash
# r06_profile.sh <group> — round 6's PMC profiles of every leg that reports traffic, at the
# tree's kernel source hash (profiles/srchash.py), in groups that fit one gpurun call:
#   c4a / c4b / c4c   the C4 legs (profile_legs.sh: kernel trace, FETCH_SIZE, TCC hit/miss)
#   small             C2 and C3: the headline count and the one-call locate
#   c5                C5: the headline count, the one-call locate and the long-pattern counts
# Output: gpurun_out/prof_legs_r06<group>_*/ (stats.json, pmc_legs.json); merge with
# profiles/merge_pmc_legs.py.  The headline count is profiled over 30 dispatches (PROF_STEPS).
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
P=$ROOT/profiles/profile_legs.sh
case "$1" in
  c4a) PROF_STEPS=30 bash "$P" r06a_c4 count && \
       bash "$P" r06a_c4 count_100m,count_u32,count_packed,count_table_steps,count_lf_loop,count_unif,count_fixed,count_rdna ;;
  c4b) bash "$P" r06b_c4 count_m32,count_m64,count_m64_steps,count_m150,count_m150_staged,count_m64_long,count_m150_long ;;
  c4c) bash "$P" r06c_c4 locate,locate_one,locate_ssa_rows,locate_m64,locate_m150,locate_m64_steps,locate_rdna,locate_ssa,wm_count,wm_lf_loop,wm_locate_ssa,learned_count,learned_lf_loop ;;
  small) PROF_STEPS=30 bash "$P" r06_c2 count,locate_one --text-bytes 99999999 --batch 1000000 && \
         PROF_STEPS=30 bash "$P" r06_c3 count,locate_one --kind bytes --text-bytes 999999999 --m 8 --batch 10000000 ;;
  c5) PROF_STEPS=20 bash "$P" r06_c5 count,locate_one,count_m64,count_m150 --text-bytes 31999999999 ;;
  *) echo "unknown group $1" >&2; exit 2 ;;
esac
