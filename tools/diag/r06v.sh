set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06v; mkdir -p $O
for o in exact window; do
  timeout -k 10 200 python -u tools/round_series.py 60 $o > $O/round_series_$o.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
for o in ("exact", "window"):
    rs = [json.loads(l) for l in open(f"gpurun_out/r06v/round_series_{o}.log") if l.startswith("{")]
    ms = {x["round"]: x["ms"] for x in rs}
    avg = lambda a, b: sum(ms[r] for r in range(a, b + 1)) / (b - a + 1)
    print(o, "rounds 5-24 %.3f  25-54 %.3f  55-59 %.3f" % (avg(5, 24), avg(25, 54), avg(55, 59)))
PY
