#!/usr/bin/env python3
"""Bytes each rank receives per frame over the collectives of the N-rank split (rtx/dist.py), and
an xGMI-time estimate: the G-buffer strip exchange (all-to-all of the rows each rank's strip-local
denoise reads), the accumulation / history / RGBA8 row all-gather (20 B/px) and the 256-B histogram
all-reduce.  On an 8-GPU MI355X node every GPU pair has its own xGMI link (7 per GPU, ~153 GB/s
each way, /opt/skills/guides/MI355X_MICROARCH.md), so a rank's receive time is bounded by the
largest share one peer sends it over one link.  Usage: tools/comm_bytes.py [W H] (default 3840 2160)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]

import torch  # noqa: E402

from rtx.dist import StripGather, denoise_rows, gbuffer_rows  # noqa: E402

LINK_GBS = 153.0


def main():
    W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (3840, 2160)
    for n in (2, 4, 8):
        need = [gbuffer_rows(H, n, r) for r in range(n)]
        worst = None
        for r in range(n):
            sg = StripGather(W, H, n, r, torch.device("cpu"))
            send, recv = sg._plan(need)
            g = sum(b for _, b in recv)
            g_link = max(b for _, b in recv)
            rows = [denoise_rows(H, n, q) for q in range(n)]
            maxr = max(b - a for a, b in rows)
            d = (n - 1) * maxr * W * 20  # padded all-gather of 20 B/px rows
            d_link = maxr * W * 20
            t = (g_link + d_link) / (LINK_GBS * 1e9) * 1e3
            if worst is None or t > worst[-1]:
                worst = (r, g, d, g_link, d_link, t)
        r, g, d, gl, dl, t = worst
        print("N=%d %dx%d: busiest rank %d receives %.1f MB G-buffer rows + %.1f MB denoise rows per frame; "
              "largest per-link share %.1f + %.1f MB -> %.3f ms at %.0f GB/s per link" %
              (n, W, H, r, g / 1e6, d / 1e6, gl / 1e6, dl / 1e6, t, LINK_GBS))


if __name__ == "__main__":
    main()
