# Single-rank eager (--graph 0, the step every W > 1 run took before round 5) vs hipGraph step
# for MLP / chunked / BERT, same box, back to back (first bullet).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_eager
export TMPDIR=/tmp
o=gpurun_out/r5_eager
for m in mlp chunked bert; do
  for g in 0 1; do
    timeout -k 10 300 python -u bench.py --model $m --graph $g --steps 20 --warmup 5 --quality-steps 0 --recall 0 --eager-compare 0 > $o/${m}_graph$g.json 2> $o/${m}_graph$g.err
    rc=$?; echo "$m graph=$g rc=$rc $(tail -1 $o/${m}_graph$g.json | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
  done
done
