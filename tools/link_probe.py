"""PCIe link probe: H2D alone, D2H alone and both directions at once between
pinned host memory and HBM (torch copies on separate streams); one JSON line."""
import json
import time

import torch


def main(gb: float = 4.0, reps: int = 3):
    dev = torch.device("cuda", 0)
    n = int(gb * (1 << 30))
    h_up = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_dn = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d_up = torch.empty(n, dtype=torch.uint8, device=dev)
    d_dn = torch.empty(n, dtype=torch.uint8, device=dev)
    h_up.fill_(1)
    d_dn.fill_(2)
    su, sd = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()

    def run(up: bool, dn: bool) -> float:
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if up:
                with torch.cuda.stream(su):
                    d_up.copy_(h_up, non_blocking=True)
            if dn:
                with torch.cuda.stream(sd):
                    h_dn.copy_(d_dn, non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    t_up, t_dn, t_both = run(True, False), run(False, True), run(True, True)
    print(json.dumps({"bytes_each_way": n, "h2d_GBps": n / t_up / 1e9, "d2h_GBps": n / t_dn / 1e9,
                      "both_s": t_both, "both_GBps_total": 2 * n / t_both / 1e9,
                      "duplex_gain": (t_up + t_dn) / t_both}))


if __name__ == "__main__":
    main()
