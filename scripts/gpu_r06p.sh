# Round 6: the routed K1 at 2 workgroups per CU (exp/rwg2: GWO_K1_ROUTE_WG=2, with register spills) against the
# product (1 per CU): the comm tests on the variant, then the 2- and 8-virtual-rank rehearsals, 2 rounds each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06p
mkdir -p $O
GWO_LIB_PATH=exp/rwg2/libgwo.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_windows.py tests/test_gpu_watermarks.py -k "comm or virtual or rank" > $O/pytest_rwg2.log 2>&1 || { tail -30 $O/pytest_rwg2.log; exit 1; }
tail -n 2 $O/pytest_rwg2.log
for rep in 1 2; do
  for L in product exp/rwg2/libgwo.so; do
    for v in 2 8; do
      tag=$(echo $L | tr '/' '_')_v$v; lp=$L; [ $L = product ] && lp=
      GWO_LIB_PATH=$lp timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-fed --comm-single --comm-virtual $v > $O/$tag.$rep.log 2>&1 || { echo FAIL $tag; tail -20 $O/$tag.$rep.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/$tag.$rep.log').read().strip().splitlines()[-1]); print('$L v$v', round(d['value']/1e9,2), 'G rec/s', round(d['ms_per_step'],4), 'ms/step', {k: round(x['total_ms']/max(x['launches'],1),4) for k,x in d.get('kernels_ms',{}).items()})"
    done
  done
done
