import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from firedancer_amd import ed25519, workload
n = 1 << 20
pub, sig, off, sz, blob = workload.sig_batch(n, 200, 1000)
chunk = int(os.environ.get("CHUNK", 1 << 17))
eng = ed25519.Engine(device=0, batch_max=chunk, blob_max=chunk * 200)
eng.verify_soa(pub[:chunk], sig[:chunk], off[:chunk], sz[:chunk], blob)
os.environ["FD_ED25519_AMD_PROFILE"] = "1"
t = time.perf_counter(); eng.verify_soa(pub, sig, off, sz, blob); print("total %.2f ms" % ((time.perf_counter() - t) * 1e3))
