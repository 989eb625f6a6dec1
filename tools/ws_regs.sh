#!/bin/bash
# Register use of one graphconv_ws_kernel instance (diagnostic build):
#   tools/ws_regs.sh FV PROD [extra -D flags]
cd "$(dirname "$0")/../graph-representation-learning_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -Wall -Wno-unused-result \
  -DGRL_DIAG -DGRL_WS_DIAG_ONE -DGRL_WS_DIAG_FV=$1 -DGRL_WS_DIAG_PROD=$2 "${@:3}" -c graphconv.hip -o /tmp/gcd.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import re,sys
txt=sys.stdin.read()
for b in txt.split('Function Name: ')[1:]:
    name=b.split()[0]
    if 'ws_kernel' not in name: continue
    g=lambda k: re.search(k+r': (\d+)',b).group(1)
    print(sys.argv[1], name[40:80], 'VGPR',g('VGPRs'),'spillV',g('VGPRs Spill'),'spillS',g('SGPRs Spill'))
" "$*"
