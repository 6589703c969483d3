#!/bin/bash
# Per-kernel VGPRs / SGPRs / spills / scratch / occupancy of mhs_kernels.hip (compiler remarks).
# usage: tools/resource_usage.sh [extra hipcc flags]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include "$@" -c $ROOT/mh-spgemm_amd/csrc/mhs_kernels.hip \
    -o /tmp/mhs_ru.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import sys, re
rows = []; cur = None
for l in sys.stdin:
    m = re.search(r'remark: Function Name: (\S+)', l)
    if m: cur = {'name': m.group(1)}; rows.append(cur); continue
    m = re.search(r'remark:\s+([\w \[\]/]+?): (\S+) \[', l)
    if m and cur is not None: cur[m.group(1).strip()] = m.group(2)
import subprocess
for r in rows:
    n = subprocess.run(['c++filt', r['name']], capture_output=True, text=True).stdout.strip()
    n = n.replace('mhs::', '').split('(')[0]
    print(f\"{n[:44]:44s} vgpr {r.get('VGPRs','?'):>4} sgpr {r.get('TotalSGPRs','?'):>4} vspill {r.get('VGPRs Spill','?'):>3} sspill {r.get('SGPRs Spill','?'):>4} scratch {r.get('ScratchSize [bytes/lane]','?'):>4} occ {r.get('Occupancy [waves/SIMD]','?'):>2}\")
"
