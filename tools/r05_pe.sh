export TMPDIR=/tmp
for rep in 1 2; do for f in "--profile-every 4" "--profile-every 1000" "--no-profile"; do
timeout -k 10 300 python3 bench.py --no-cpu --no-host-path --no-config3 --no-config4 --no-config5 --no-wide --no-pmc --steps 100 $f > gpurun_out/pe.json 2>/dev/null || exit 1
python3 -c "
import json,sys
d=json.loads(open('gpurun_out/pe.json').read().strip().splitlines()[-1])
print(sys.argv[1], round(d['ms_per_step'],4), d['parity'])
" "$f"
done; done
