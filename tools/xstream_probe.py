#!/usr/bin/env python3
"""Cost of a cross-stream dependency on this GPU (tools only): a chain of small
kernels alternating between two streams, each step waiting for the other
stream's last kernel through an event, against the same chain on one stream;
plus the overlap of two independent chains on two streams.  Prints one JSON line."""
import json
import time

import torch


def main():
    dev = torch.device("cuda:0")
    x = torch.zeros(1 << 16, device=dev)
    y = torch.zeros(1 << 16, device=dev)
    big = torch.zeros(1 << 26, device=dev)  # 256 MiB: ~60 us of streaming per add
    s1, s2 = torch.cuda.current_stream(), torch.cuda.Stream()
    n = 200

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e6

    def one_stream():
        for _ in range(n):
            x.add_(1)
            y.add_(1)

    def alternating():
        for _ in range(n):
            x.add_(1)
            e = torch.cuda.Event()
            e.record(s1)
            s2.wait_event(e)
            with torch.cuda.stream(s2):
                y.add_(1)
            f = torch.cuda.Event()
            f.record(s2)
            s1.wait_event(f)

    def big_one():
        for _ in range(n // 10):
            big.add_(1)
            x.add_(1)

    def big_two():  # a small kernel on s2 beside each big one on s1, joined every step
        for _ in range(n // 10):
            e = torch.cuda.Event()
            e.record(s1)
            s2.wait_event(e)
            big.add_(1)
            with torch.cuda.stream(s2):
                x.add_(1)
            f = torch.cuda.Event()
            f.record(s2)
            s1.wait_event(f)

    r = {"one_stream_us_per_step": round(timed(one_stream), 2),
         "alternating_two_streams_us_per_step": round(timed(alternating), 2),
         "big_plus_small_one_stream_us": round(timed(big_one) * 10, 2),
         "big_plus_small_two_streams_joined_us": round(timed(big_two) * 10, 2)}
    print(json.dumps(r))


if __name__ == "__main__":
    main()
