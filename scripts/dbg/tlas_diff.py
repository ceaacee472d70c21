"""Find pixels where the TLAS and the linear object loop disagree at full size, and check the
rows against the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "raytracer-795_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402
import rtg  # noqa: E402
from rtg import scenegen  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
sc = scenegen.spheres(1920, 1080, spp=spp)
out = {}
for tl in (1, 2):
    with rtg.Renderer(sc, device=0, tlas=tl) as r:
        out[tl] = (r.render(0), r.stats())
a, sa = out[1]
b, sb = out[2]
print({k: (sa[k], sb[k]) for k in ("primary_rays", "secondary_rays", "shadow_rays")})
d = np.any(a.view(np.int32) != b.view(np.int32), axis=2)
ys, xs = np.nonzero(d)
print("differing pixels", len(ys))
for y, x in list(zip(ys, xs))[:20]:
    print(y, x, a[y, x], b[y, x])
rows = sorted(set(ys.tolist()))[:3]
o = pyoracle.Oracle(sc)
for y in rows:
    ref = o.render(0, nthreads=16, row_begin=y, row_end=y + 1)[0]
    xs_ = np.nonzero(d[y])[0]
    for x in xs_[:5]:
        print("row", y, "x", x, "oracle", ref[y, x], "linear", a[y, x], "tlas", b[y, x])
