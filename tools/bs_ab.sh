# strong-scaling shares (tools/band_share_time.py) under environment variants
for v in "-" "RT_SORT=shadow" "RT_INLINE_SHADOW=0"; do echo "$v"; if [ "$v" = "-" ]; then timeout -k 10 100 python tools/band_share_time.py 3; else env $v timeout -k 10 100 python tools/band_share_time.py 3; fi; done > gpurun_out/bs3.log 2>&1
