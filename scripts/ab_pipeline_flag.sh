cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2 3; do
  for P in 0 1; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ode-calls 0 --f32-steps 0 --pointwise-steps 0 --pipeline $P > gpurun_out/pp.json 2> gpurun_out/pp.err || exit 1
    echo "$r pipeline=$P $(python -c "import json;d=json.loads(open('gpurun_out/pp.json').read().strip().splitlines()[-1]);r=d['roofline'];print(f\"ms_per_step={d['ms_per_step']:.3f} sampler_ms={r.get('sampler_ms_per_step',0):.3f} pc_us={r['avg_launch_us']:.2f}\")")"
  done
done
