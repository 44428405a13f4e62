# Per-step host timestamps of the default bench (27 cameras) over a long
# window: does the step time drift over the run (warm-up, clocks)?
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r05steps}
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 3 --step-times > $O/s200.json 2> $O/s200.err || { tail $O/s200.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/d1.json 2> $O/d1.err || { tail $O/d1.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 20 > $O/w20.json 2> $O/w20.err || { tail $O/w20.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/${TAG:-r05steps}/s200.json".replace("${TAG:-r05steps}", __import__("os").environ.get("TAG", "r05steps"))))
h = d["host_step_ms"]
for a in range(0, len(h), 20):
    seg = h[a:a + 20]
    print(f"steps {a:3d}-{a + len(seg) - 1:3d}: mean {sum(seg) / len(seg):.3f} ms")
for n in ("d1", "w20"):
    e = json.load(open(f"gpurun_out/{__import__('os').environ.get('TAG', 'r05steps')}/{n}.json"))
    print(n, e["ms_per_step"], e["steps"], e["warmup"])
PY
