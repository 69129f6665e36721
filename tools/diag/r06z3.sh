set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06z3; mkdir -p $O
for n in 65536 131072 262144 372736; do
  timeout -k 10 300 python -u tools/big_mesh.py --nodes $n --rounds 6 --out $O/big_$n.json > $O/big_$n.log 2>&1 || { tail -5 $O/big_$n.log; exit 1; }
  tail -2 $O/big_$n.log
done
