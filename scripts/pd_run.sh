set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${PD_TAG:-pd}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-stats --no-render-api"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $B > $O/trace.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1
cd $R
python3 scripts/per_dispatch.py $O | tee $O/per_dispatch.txt
MFX_DIAG_ITER=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-render-api --no-stats > $O/diag.json 2> $O/diag.txt
grep "gen 0" $O/diag.txt | tail -4
MFX_RAY_QUEUE=0 MFX_DIAG_ITER=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-render-api --no-stats > $O/diag_off.json 2> $O/diag_off.txt
grep "gen 0" $O/diag_off.txt | tail -4
