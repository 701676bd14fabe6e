"""Kernel-time probe of the pooled DSM stage on one resident 2^20 batch
(k_dsmp forced), for rocprofv3 --kernel-trace --stats runs of A/B builds
(FD_AMD_LIB).  Verdicts are not checked: an A/B build may void them.
    rocprofv3 --kernel-trace --stats -d out -- python3 tools/kai_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519, hip, workload  # noqa: E402

n = 1 << 20
d = [hip.DeviceBuffer.from_array(a) for a in workload.sig_batch(n, 200, 12)]
err, ws = hip.DeviceBuffer(n), hip.DeviceBuffer(ed25519.workspace_footprint(n))
ed25519.select_dsm_kernel("k_dsmp")
st = hip.Stream()
for _ in range(4):
    ed25519.verify_dev(n, *[x.ptr for x in d], err.ptr, ws.ptr, st.handle)
st.synchronize()
print("ok")
