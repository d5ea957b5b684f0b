# GPU call script (gpurun): every BASELINE config on the round's final build (one line each; self-checked).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${CFG_TAG:-r4c}; mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -8 $O/$name.log; echo "stopping after $name (rc $rc)"; exit $rc; fi
  grep -o '"value": [0-9.]*\|"us_per_generation[a-z_]*": [0-9.]*\|"ok": [a-z]*' $O/$name.log | head -6 | tr '\n' ' '; echo
}
# config 1: the reference's 100^2 torus, .NET Random (GameOfLifeDriver.fs:9-19), 100 generations in one call
step c1 120 python bench.py --init dotnet-mod2 --seed 42 --width 100 --height 100 --generations 100 --gens-per-step 100 --steps 20 --warmup 3
# config 2: 4096^2 torus, 1000 generations
step c2 120 python bench.py --init dotnet-mod2 --seed 42 --width 4096 --height 4096 --generations 1000 --gens-per-step 1000 --steps 3 --warmup 1
# config 3: the whole 10k-generation job at 65536^2 (834 passes of 12)
step c3_job 400 python bench.py --gpus 1 --warmup 5 --no-cpu-baseline
# config 4's board on one GPU (262144^2, 16 GiB double-buffered), 20 passes
step c4_1gpu 400 python bench.py --gpus 1 --board 262144 --steps 20 --warmup 3 --no-cpu-baseline --handle-parts 0
# config 5: gun + R-pentomino, 4096^2 torus (cooperative pass) and 256^2 bounded (rows-on-lanes), 100k generations
step c5_4096 200 python bench.py --init rle:gosper-gun@1000,1000+r-pentomino@3000,3000 --width 4096 --height 4096 --generations 100000 --gens-per-step 50000 --steps 1 --warmup 1
step c5_256 120 python bench.py --init rle:gosper-gun@10,10+r-pentomino@180,150 --width 256 --height 256 --boundary bounded --generations 100000 --gens-per-step 50000 --steps 1 --warmup 1
