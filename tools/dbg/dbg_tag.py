import sys, os, hashlib
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import _golden
from firedancer_amd import ed25519, hip, tango
g = _golden.load_vectors()
sel = [i for i in range(len(g)) if g.expect[i] == 0][:70]
n = len(sel)
msgs = [g.msg(i) for i in sel]
off = np.cumsum([0] + [len(m) for m in msgs[:-1]]).astype(np.uint32)
blob = np.frombuffer(b"".join(msgs) + b"\0" * 16, np.uint8)
d = {k: hip.DeviceBuffer.from_array(v) for k, v in dict(pub=g.pub[sel], sig=g.sig[sel], off=off, sz=g.msg_sz[sel], blob=blob).items()}
err = hip.DeviceBuffer(n); ws = hip.DeviceBuffer(ed25519.workspace_footprint(n)); st = hip.Stream()
ed25519.verify_dev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, err.ptr, ws.ptr, st.handle)
st.synchronize()
N = 128
al = lambda x: (x + 255) & ~255
o = 0
for sz in (512 * N, 4 * N, 120 * N, 80 * N, 1536 * N, 12 * N):
    o = al(o + sz)
raw = ws.to_array(np.uint8, ed25519.workspace_footprint(n))
tags = raw[o:o + 8 * n].view(np.uint64)
exp = [int.from_bytes(hashlib.sha512(bytes(g.sig[i][:32]) + bytes(g.pub[i]) + g.msg(i)).digest()[:8], "little") for i in sel]
print("ws tags match:", [int(t) for t in tags[:3]], exp[:3], all(int(a) == b for a, b in zip(tags, exp)))
print("err", err.to_array(np.int8, n)[:10])
