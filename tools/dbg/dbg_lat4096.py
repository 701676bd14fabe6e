"""One 4096-signature device-resident batch, repeated: the latency kernels
(k_front + k_dsm4) for PMC passes."""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from firedancer_amd import ed25519, hip, workload
n = 4096
pub, sig, off, sz, blob = workload.sig_batch(n, 200, 7)
d = {k: hip.DeviceBuffer.from_array(v) for k, v in dict(pub=pub, sig=sig, off=off, sz=sz, blob=blob).items()}
err = hip.DeviceBuffer(n); ws = hip.DeviceBuffer(ed25519.workspace_footprint(n)); st = hip.Stream()
for r in range(20):
    ev = [hip.Event() for _ in range(4)]
    ed25519.verify_dev_ev(n, d["pub"].ptr, d["sig"].ptr, d["off"].ptr, d["sz"].ptr, d["blob"].ptr, err.ptr, ws.ptr, st.handle, ev)
    st.synchronize()
print("k_dsm4 ms", ev[2].elapsed_ms(ev[3]))
