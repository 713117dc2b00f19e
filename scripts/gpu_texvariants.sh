set -u
cd $GRAFT_REPO_ROOT
for v in variants/*.so; do
  timeout -k 10 200 python -c "
import sys; sys.argv=['x']; import various_image_processings_amd._lib as L; L.LIB_PATH='$v'
import numpy as np, torch; sys.path.insert(0,'.')
import various_image_processings_amd as vip
from oracle import oracle as o
img=o.random_image(203,131); d=torch.from_numpy(img).cuda(); out=torch.empty_like(d)
vip.CudaBilateralTextureFilter(203,131,5,2).execute(d,out)
print('$v texture parity', np.array_equal(out.cpu().numpy(), o.texture(img,5,2)))
" || exit 1
done
timeout -k 10 300 python scripts/variant_bench.py various_image_processings_amd/libvip_hip.so variants/*.so
