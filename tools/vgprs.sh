#!/bin/bash
# VGPRs / occupancy / LDS of every kernel in libbkdigest (device-only compile, no GPU needed).
cd /tmp && hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --cuda-device-only -c -I /root/repo/include \
  ${BKD_EXTRA_FLAGS} /root/repo/bookkeeper_amd/csrc/bkdigest.hip -o /tmp/bk_dev.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/{n=$0; sub(/.*Function Name: /,"",n); sub(/ \[-R.*/,"",n)} /VGPRs:/ && !/Spill/{v=$0; sub(/.*VGPRs: /,"",v); sub(/ \[.*/,"",v)} /Occupancy/{o=$0; sub(/.*SIMD\]: /,"",o); sub(/ \[.*/,"",o)} /LDS Size/{l=$0; sub(/.*block\]: /,"",l); sub(/ \[.*/,"",l); print v, o, l, n}' | c++filt
