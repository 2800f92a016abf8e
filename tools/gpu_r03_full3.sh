# round 3 evidence: the whole -m gpu suite, then every bench config once (CPU baselines included)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03z; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > $O/pytest_all.log 2>&1 || { echo "FAIL gpu tests"; tail -40 $O/pytest_all.log; exit 1; }
echo "gpu tests ok: $(tail -1 $O/pytest_all.log)"
for c in "northstar:" "reference:--semantics reference" "tree:--order tree" "c2:--config c2" "c3:--config c3" \
         "gmapping:--config gmapping" "plicp:--config plicp" "karto:--config karto" "karto_loop:--config karto_loop"; do
  name=${c%%:*}; args=${c#*:}
  timeout -k 10 400 python3 bench.py $args > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  echo "done $name"
done
