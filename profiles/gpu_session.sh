#!/bin/bash
# gpu_session.sh <tag> <step> [<step> ...] — one gpurun session on the MI355X box.
#
# Replaces round 1's one-off session2_*.sh wrappers.  Every step runs under its own
# time limit; the first failing step ends the session (no retries).  Outputs go to
# gpurun_out/<tag>_<step name>.{json,err,log}; summaries worth keeping are copied to
# profiles/rNN/ by hand.  A step is one quoted word list:
#
#   "tests [pytest -k expr]"       the -m gpu suite (or the tests matching expr)
#   "smoke"                        __graft_entry__.smoke()
#   "bench <cfg> [VAR=val ...] [bench.py args ...]"
#                                  one bench.py line (<name>.json; every leg in <name>.full.json);
#                                  <cfg> picks the BASELINE config:
#                                  c2 (100 MB DNA, 1 M 20-mers), c3 (1 GB bytes, 10 M 8-mers),
#                                  c4 (the default), c5 (32 GB DNA); VAR=val set the engine's
#                                  environment switches (CS_FM_ENGINE=wavelet, CS_FM_COUNT_U=1, ...)
#   "prof <cfg> <leg,leg,...> [bench.py args ...]"
#                                  profile_legs.sh passes (kernel trace, FETCH_SIZE, L2)
#   "gather <GB> [<GB> ...]"       profiles/microbench/gather_bench over tables of these sizes
#   "phases [VAR=val ...]"         profiles/scripts/locate_phases.py (C4 locate phases)
#
# e.g.  bash profiles/gpu_session.sh r02 "tests" "smoke" "bench c4" "prof c3 count"
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
TAG=$1
shift
OUT=gpurun_out
mkdir -p $OUT

cfg_args() {
  case $1 in
    c2) echo "--text-bytes 99999999 --batch 1000000" ;;
    c3) echo "--kind bytes --text-bytes 999999999 --m 8 --batch 10000000" ;;
    c4) echo "" ;;
    c5) echo "--text-bytes 31999999999" ;;
    *) echo "unknown config $1" >&2; return 1 ;;
  esac
}

n=0
for STEP in "$@"; do
  n=$((n + 1))
  read -r -a W <<< "$STEP"
  KIND=${W[0]}
  ENVS=()
  ARGS=()
  for x in "${W[@]:1}"; do
    if [[ $x =~ ^[A-Z_][A-Z0-9_]*=.* ]]; then ENVS+=("$x"); else ARGS+=("$x"); fi
  done
  NAME="${TAG}_${n}_${KIND}"
  echo "[gpu_session] step $n: $STEP" >&2
  case $KIND in
    tests)
      K=()
      [ ${#ARGS[@]} -gt 0 ] && K=(-k "${ARGS[*]}")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=80 \
        "${K[@]}" > $OUT/$NAME.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/$NAME.log 2>&1 ;;
    bench)
      C=$(cfg_args "${ARGS[0]}") || exit 1
      NAME="${NAME}_${ARGS[0]}"
      env "${ENVS[@]}" timeout -k 10 600 python -u bench.py $C --legs-out $OUT/$NAME.full.json "${ARGS[@]:1}" > $OUT/$NAME.json 2> $OUT/$NAME.err ;;
    prof)
      C=$(cfg_args "${ARGS[0]}") || exit 1
      env "${ENVS[@]}" timeout -k 10 900 bash profiles/profile_legs.sh "${TAG}_${ARGS[0]}" "${ARGS[1]}" $C \
        "${ARGS[@]:2}" > $OUT/$NAME.log 2>&1 ;;
    gather)
      for g in "${ARGS[@]}"; do
        timeout -k 10 120 profiles/microbench/gather_bench "$g" 256 > $OUT/${NAME}_${g}g.txt 2>&1 || exit 1
      done ;;
    phases)
      env "${ENVS[@]}" timeout -k 10 300 python -u profiles/scripts/locate_phases.py > $OUT/$NAME.json 2> $OUT/$NAME.err ;;
    *)
      echo "unknown step $KIND" >&2; exit 2 ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "[gpu_session] step $n ($STEP) failed with status $rc: session ends here" >&2
    exit $rc
  fi
done
