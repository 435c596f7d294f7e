#!/bin/bash
# lstm.hip alone, one .so per variant (name:flags ...), for tools/lstm_time.py A/B runs
cd "$(dirname "$0")/.." || exit 1
K=dinunet_implementations_amd/csrc/kernels
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; [ "$flags" = "$spec" ] && flags=""
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=fast -fno-slp-vectorize \
    -Wno-unused-result $flags -I $K $K/lstm.hip -o tools/_variants/lstm_$name.so &
done
wait
ls tools/_variants
