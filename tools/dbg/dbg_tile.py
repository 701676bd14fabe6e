import sys, os, hashlib
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import _golden, test_tile_gpu as T
from firedancer_amd import tango
g = _golden.load_vectors()
pub, sig, msgs, verdict = T._pool(g)
order = np.arange(6)
mc_in, dc, chunks, sizes, ts = T._feed(pub, sig, msgs, order, 64)
mc_out = tango.mcache_new(64)
tile = tango.VerifyTile(0, batch_max=4, tcache_depth=16)
diag, lat = tile.run(mc_in, dc, 0, mc_out, 0, 6, lat_max=6)
print(diag)
print(mc_in[:6])
print(mc_out[:6])
exp, ha, sv = T._model(pub, sig, msgs, order, verdict, 16)
print(exp, verdict[:6])
