set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2h; mkdir -p $O; cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify > $O/b20_launch_$i.json 2>>$O/err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify --kernel-events region > $O/b20_region_$i.json 2>>$O/err || exit 2
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify --settle-ms 0 > $O/b20_nosettle.json 2>>$O/err || exit 3
timeout -k 10 300 python bench.py --steps 600 --warmup 10 --no-cpu-baseline --no-verify > $O/b600_launch.json 2>>$O/err || exit 4
timeout -k 10 300 python bench.py --steps 600 --warmup 10 --no-cpu-baseline --no-verify --kernel-events region > $O/b600_region.json 2>>$O/err || exit 5
for f in $O/b*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])"; done
