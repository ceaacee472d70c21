import sys, numpy as np
sys.path[:0] = ['raytracer-795_amd', 'oracle']
import rtg, pyoracle
from rtg import scenegen as G, _abi as A
sc = G.furnace(16, 12, spp=16, flags=A.PT_NEE)
o = pyoracle.Oracle(sc)
ref = o.render(0)[0]
with rtg.Renderer(sc, device=0) as r:
    for trav in (0, 1):
        img = r.render(0, traversal=trav)
        print("trav", trav, img[4:8, 6:10].reshape(-1, 3).mean(0), "oracle", ref[4:8, 6:10].reshape(-1, 3).mean(0), r.stats()["shadow_rays"])
    dirs = np.array([[0, 0, 1], [0, 1, 0], [1, 0, 0], [0.3, 0.4, 0.866]], np.float32)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    org = np.array([[0, 0, 1.002]] * 4, np.float32)
    print("gpu", r.trace(org, dirs))
    print("orc", o.trace(org, dirs))
