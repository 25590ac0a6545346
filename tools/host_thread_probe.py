"""Host thread scaling of the replicate-file work (crc32 + sha256 + write) on this box."""
import concurrent.futures as cf
import hashlib
import os
import tempfile
import time
import zlib

import numpy as np

data = [np.random.rand(20000).astype(np.float32).tobytes() for _ in range(900)]
d = tempfile.mkdtemp()
print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for nt in (1, 4, 8, 16):
    t = time.perf_counter()
    with cf.ThreadPoolExecutor(nt) as ex:
        list(ex.map(lambda b: (zlib.crc32(b), hashlib.sha256(b).hexdigest()), data))
    t1 = time.perf_counter() - t

    def w(i):
        p = os.path.join(d, f"f{nt}_{i}.tmp")
        with open(p, "wb") as fh:
            fh.write(data[i])
        os.replace(p, p[:-4] + ".npz")
    t = time.perf_counter()
    with cf.ThreadPoolExecutor(nt) as ex:
        list(ex.map(w, range(900)))
    print(f"threads {nt}: crc+sha {t1:.3f} s, write+rename {time.perf_counter() - t:.3f} s")
