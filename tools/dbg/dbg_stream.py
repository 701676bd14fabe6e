import sys, os, json
sys.path.insert(0, os.getcwd())
import numpy as np
from firedancer_amd import tango, workload
pub, sig, off, sz, blob = workload.sig_batch(8192, 200, 1)
for bmax, rate, nf in ((256, 2000, 2000), (256, 20000, 20000), (256, 100000, 50000), (4096, 100000, 50000), (4096, 1000000, 300000)):
    r = tango.bench_stream(0, bmax, 0, pub, sig, off, sz, blob, nf, rate=rate)
    print(bmax, rate, json.dumps({k: round(v, 1) for k, v in r.items()}))
