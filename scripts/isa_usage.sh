# Per-variant VGPRs / scratch / occupancy of the path kernels (host-side, no GPU): bash scripts/isa_usage.sh [extra hipcc flags]
set -e
cd "$(dirname "$0")/../raytracer-weekend_amd"
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -fno-gpu-rdc -fno-slp-vectorize \
  -mllvm -amdgpu-atomic-optimizer-strategy=None -mllvm -amdgpu-sched-strategy=max-ilp --cuda-device-only -S csrc/rtw_kernel.hip -o /tmp/isa/k.s "$@" 2>/dev/null
python3 - <<'PY'
import re
txt = open('/tmp/isa/k.s').read()
for m in re.finditer(r'^(_ZN3rtw3dev11path_kernelILb0E\S*?):\s*;', txt, re.M):
    name = m.group(1); i = txt.find('.Lfunc_end', m.end()); seg = txt[i:i + 3000]
    g = lambda k: re.search(k + r':\s*(\d+)', seg).group(1)
    body = txt[m.end():i]
    nv = sum(1 for l in body.splitlines() if l.strip().startswith('v_'))
    print(name[len('_ZN3rtw3dev11path_kernelI'):-len('EEEvNS_10RenderArgsE')], 'vgpr', g('NumVgprs'), 'scratch', g('ScratchSize'), 'occ', g('Occupancy'), 'static_valu', nv)
PY
