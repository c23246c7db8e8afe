#!/bin/bash
# Static VALU mix (tools/isa_count.py, priced with the measured issue costs of DESIGN.md §4) of the kernels bench.py
# reports a roofline for -> profiles/<tag>_isa_mix.json (bench.py: roofline.valu_cycle_weighted).
set -eu
TAG=${1:-r03}
cd "$(dirname "$0")/.."
T=$(mktemp -d)
for f in nmt_kernels rs_kernels rs16_kernels; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -o $T/$f.s celestia-app_amd/csrc/$f.hip 2>/dev/null
  python3 tools/isa_count.py $T/$f.s "leaf_hash|nmt_levels|dah_kernel|rs_encode" --json $T/$f.json > /dev/null
done
python3 - "$T" "$TAG" <<'PY'
import json, sys
t, tag = sys.argv[1], sys.argv[2]
out = {}
for f in ("nmt_kernels", "rs_kernels", "rs16_kernels"):
    out.update(json.load(open(f"{t}/{f}.json")))
json.dump(out, open(f"profiles/{tag}_isa_mix.json", "w"), indent=1, sort_keys=True)
print("wrote", f"profiles/{tag}_isa_mix.json", len(out), "kernels")
PY
rm -rf $T
