# PC sampling of the north-star bench (rocprofv3 beta): tools/pcsample.sh <tag> <method> <unit> <interval>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; M=${2:-stochastic}; U=${3:-cycles}; I=${4:-1048576}
export TMPDIR=/tmp; O=$R/gpurun_out/pcs_$T; mkdir -p $O; cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/list.txt 2>&1; grep -i -B2 -A12 "pc.sampl\|PC Sampl" $O/list.txt | head -60
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U --pc-sampling-interval $I \
   -d $O/run -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-copy-probe --steps 3 --warmup 1 > $O/run.log 2>&1
echo "rc $?"; tail -5 $O/run.log; ls -la $O/run/* | head
