"""Device -> host copy of a large tensor: pageable ``.cpu()`` vs utils.transfer.to_host
(pinned double-buffered chunks, threaded unpack).  Prints one JSON line per size."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cnmf_torch_amd.utils.transfer import to_host  # noqa: E402


def main():
    for gb in (0.5, 4.0):
        n = int(gb * (1 << 30) / 4) // 2000 * 2000
        t = torch.rand(n, device="cuda").view(-1, 2000)
        torch.cuda.synchronize()
        res = {}
        for name, fn in (("pageable_cpu", lambda: t.cpu().numpy()), ("to_host", lambda: to_host(t))):
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter()
                a = fn()
                best = min(best, time.perf_counter() - t0)
                del a
            res[name] = round(best, 4)
        b = to_host(t)
        ok = bool(np.array_equal(b, t.cpu().numpy()))
        print(json.dumps({"gb": gb, "seconds": res, "gbps": {k: round(gb / v, 2) for k, v in res.items()},
                          "bitwise_equal": ok}), flush=True)
        del t, b


if __name__ == "__main__":
    main()
