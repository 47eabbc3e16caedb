# GPU box: bench lines named on the command line (LINES="name:args;name:args"), each under its
# own time limit, outputs under gpurun_out/$TAG; stops at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-lines}
mkdir -p $O
IFS=';' read -ra L <<< "$LINES"
for item in "${L[@]}"; do
  name=${item%%:*}; args=${item#*:}
  timeout -k 10 ${LINE_TIMEOUT:-300} python bench.py $args > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  python scripts/bench_line.py $O/$name.json $name
done
echo done
