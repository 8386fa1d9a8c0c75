# Helper sourced by the GPU scripts: `step NAME SECONDS CMD...` runs one GPU step under its
# own time limit, logs to gpurun_out/NAME.log, and ends the whole call after a time limit,
# abort or crash (rc 124/134/137/139 or >128) — an ordinary failure (rc 1, e.g. a failed
# test) is recorded and the next step still runs.
step() {
  local name=$1 secs=$2
  shift 2
  echo "[step] $name start $(date +%T)"
  timeout -k 10 $secs "$@" > $GRAFT_REPO_ROOT/gpurun_out/$name.log 2>&1
  local rc=$?
  echo "[step] $name rc=$rc $(date +%T)"
  if [ $rc -ge 124 ]; then
    echo "[step] $name ended with rc=$rc: stopping this call"
    exit $rc
  fi
  return 0
}
