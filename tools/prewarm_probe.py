"""Wall time of utils.prewarm in a fresh process: its groups on one thread each or all on
one thread (``--serial``), from start() to wait().  One JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cnmf_torch_amd.utils import prewarm  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--serial", action="store_true")
    a = ap.parse_args()
    torch.zeros(1, device="cuda").sum().item()          # context up first
    t0 = time.perf_counter()
    prewarm.start(torch.device("cuda", 0), parallel=not a.serial)
    prewarm.wait()
    print(json.dumps({"parallel": not a.serial, "prewarm_s": round(time.perf_counter() - t0, 3),
                      "errors": prewarm.errors}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
