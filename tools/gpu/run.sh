#!/bin/bash
# Parameterised GPU pass: one gpurun call = one TAG and a list of steps.
#
#   bash tools/gpu/run.sh TAG 'name|seconds|command' ['name|seconds|command' ...]
#
# Each step runs under its own `timeout -k 10 <seconds>`, writes stdout+stderr to
# gpurun_out/TAG/<name>.log and prints its last line.  The first failing step ends the
# call (no later GPU step runs after a fault, abort or time limit).  Named shortcuts:
#   pytest          every GPU test (one process)
#   smoke           __graft_entry__.smoke()
#   bench:ARGS      python bench.py ARGS       (ARGS with '_' for spaces)
#   prof:ARGS       rocprofv3 --kernel-trace --stats of bench.py ARGS (-> TAG/prof_<n>/)
# e.g.  bash tools/gpu/run.sh r6a 'b20|120|python bench.py --steps 20' prof:--steps_10
export TMPDIR=/tmp
tag=$1
shift
out=gpurun_out/$tag
mkdir -p "$out"
i=0
for spec in "$@"; do
  i=$((i + 1))
  case "$spec" in
    pytest) name=pytest; secs=900
      cmd="python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" ;;
    smoke) name=smoke; secs=200; cmd="python -c 'import __graft_entry__ as g; g.smoke()'" ;;
    bench:*) a=${spec#bench:}; name=bench$i; secs=300; cmd="python bench.py ${a//_/ }" ;;
    prof:*) a=${spec#prof:}; name=prof$i; secs=240
      cmd="rocprofv3 --kernel-trace --stats -d $out/prof_$i -o run -- python3 bench.py ${a//_/ }" ;;
    *) name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|} ;;
  esac
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  tail -n 1 "$out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then
    echo "STEP $name FAILED rc=$rc"
    tail -n 30 "$out/$name.log"
    exit $rc
  fi
done
