#!/bin/bash
# Register / occupancy report of the kernels of one HIP source:
#   tools/vgprs.sh csrc/attention.hip [name-regex]
cd "$(dirname "$0")/../graph-neural-pde_amd" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 --cuda-device-only -c "$1" -o /tmp/vgprs_probe.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import sys, re
pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur, row = None, {}
def flush():
    if cur and (pat is None or pat.search(cur)):
        print('%-90s vgpr %4s occ %2s scratch %s' % (cur[:90], row.get('VGPRs'), row.get('Occupancy [waves/SIMD]'), row.get('ScratchSize [bytes/lane]')))
for line in sys.stdin:
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        flush(); cur, row = m.group(1), {}; continue
    m = re.search(r'(VGPRs|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\d+)', line)
    if m: row[m.group(1)] = m.group(2)
flush()
" "${2:-}"
