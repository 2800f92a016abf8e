#!/bin/bash
# One GPU session, steps chosen by name, results under gpurun_out/<tag>/ (each step under its own limit,
# the session stops at the first failure):
#   tools/gpu_session.sh <tag> <step>...
#   cold     the driver's exact bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5) -> cold.json
#            (run it FIRST to time a cold box: no GPU process before it)
#   pytest   python -m pytest tests -m gpu                                                        -> pytest.log
#   pytestab:<lib>[:<files>]  the GPU tests against lib/ab/libslam2d_<lib>.so                    -> pytest_<lib>.log
#   uclk     tools/clk_update.py on lib/ab/libslam2d_uclk.so (the update's tile-loop phase split) -> uclk.json
#   mclk     tools/clk_match.py on lib/ab/libslam2d_mclk.so (the match's GN-step phase split)          -> mclk.txt
#   smoke    __graft_entry__.smoke()                                                              -> smoke.log
#   warm     the driver's bench command again                                                     -> warm.json
#   bench:<name>:<args>   bench.py <args> (commas become spaces)                                   -> <name>.json
#   ab:<lib>,<lib>...     tools/ab_bench.sh over lib/ab/libslam2d_<lib>.so ("main" = the product library)
#   pmc:<lib>,<lib>...    tools/pmc_ab.sh counter passes per variant (PMC_SETS="set;set" to choose) -> pmc.txt
#   prof:<name>:<args>    tools/profile_gpu.sh <tag>_<name> <args>
set -o pipefail
T=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$T
mkdir -p "$O"
cd "$R"
for step in "$@"; do
  case "$step" in
    cold|warm)
      timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/$step.json" 2> "$O/$step.err" \
        || { echo "FAIL $step"; tail -20 "$O/$step.err"; exit 1; }
      python3 tools/ab_summary.py --line "$O/$step.json" ;;
    pytest)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 \
        || { echo "FAIL pytest"; tail -30 "$O/pytest.log"; exit 1; }
      tail -2 "$O/pytest.log" ;;
    pytestab:*)
      # pytestab:<lib>[:<test files, commas>]  the GPU tests against lib/ab/libslam2d_<lib>.so
      rest=${step#pytestab:}; lib=${rest%%:*}; files=${rest#*:}; [ "$files" = "$rest" ] && files=tests
      SLAM2D_LIB=$R/creating-2d-laser-slam-from-scratch_amd/lib/ab/libslam2d_$lib.so timeout -k 10 900 \
        python3 -u -m pytest ${files//,/ } -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_$lib.log" 2>&1 \
        || { echo "FAIL pytestab $lib"; tail -30 "$O/pytest_$lib.log"; exit 1; }
      echo "pytest $lib: $(tail -1 "$O/pytest_$lib.log")" ;;
    uclk)
      # the update kernel's tile-loop phase split (tools/build_diag.py uclk; built beforehand into lib/ab/)
      SLAM2D_LIB=$R/creating-2d-laser-slam-from-scratch_amd/lib/ab/libslam2d_uclk.so timeout -k 10 300 \
        python3 tools/clk_update.py > "$O/uclk.json" 2> "$O/uclk.err" || { echo "FAIL uclk"; tail -20 "$O/uclk.err"; exit 1; }
      cat "$O/uclk.json" ;;
    mclk)
      # the match's Gauss-Newton step phase split (tools/build_diag.py mclk; built beforehand into lib/ab/)
      SLAM2D_LIB=$R/creating-2d-laser-slam-from-scratch_amd/lib/ab/libslam2d_mclk.so timeout -k 10 300 \
        python3 tools/clk_match.py > "$O/mclk.txt" 2> "$O/mclk.err" || { echo "FAIL mclk"; tail -20 "$O/mclk.err"; exit 1; }
      cat "$O/mclk.txt" ;;
    smoke)
      timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { echo "FAIL smoke"; tail -20 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" ;;
    bench:*)
      rest=${step#bench:}; name=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      timeout -k 10 300 python3 bench.py ${args//,/ } > "$O/$name.json" 2> "$O/$name.err" \
        || { echo "FAIL $step"; tail -20 "$O/$name.err"; exit 1; }
      python3 tools/ab_summary.py --line "$O/$name.json" ;;
    ab:*)
      libs=${step#ab:}
      bash tools/ab_bench.sh "$T" ${libs//,/ } || exit 1 ;;
    pmc:*)
      # pmc:<lib>,<lib>...  tools/pmc_ab.sh counters per variant (PMC_SETS from the environment, else its defaults)
      libs=${step#pmc:}
      timeout -k 10 900 bash tools/pmc_ab.sh "$T" ${libs//,/ } > "$O/pmc.txt" 2>&1 || { echo "FAIL pmc"; tail -20 "$O/pmc.txt"; exit 1; }
      cat "$O/pmc.txt" ;;
    prof:*)
      rest=${step#prof:}; name=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      bash tools/profile_gpu.sh "${T}_$name" ${args//,/ } || { echo "FAIL $step"; exit 1; } ;;
    calib)
      # WRITE_SIZE / FETCH_SIZE calibration on the update's store shapes (tools/probes/write_calib.hip, built
      # beforehand into tools/probes/build/): one plain run, then one --pmc pass per counter
      B=$R/tools/probes/build/write_calib
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 "$B" > "$O/expected.json" 2> "$O/calib.err" \
        && timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/write" -o run --output-format csv -- "$B" > "$O/w.log" 2>&1 \
        && timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/fetch" -o run --output-format csv -- "$B" > "$O/f.log" 2>&1) \
        || { echo "FAIL calib"; tail -20 "$O/calib.err" "$O/w.log" "$O/f.log" 2>/dev/null; exit 1; }
      python3 tools/write_calib.py "$O" "$O/write_calib" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
