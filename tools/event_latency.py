"""Cross-queue event hand-off latency on this runtime: queue 1 runs a ~1 ms GEMM chain and
records an event; queue 2 (idle) waits on it and records a timed event. Prints the delay
between queue 1's timed marker (right after the event) and queue 2's, per event flavour.
    python tools/event_latency.py"""
import torch


def run(timing_evt, reps=20):
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda")
    b = torch.randn(4096, 4096, device="cuda")
    d = []
    for _ in range(reps):
        e = torch.cuda.Event(enable_timing=timing_evt)
        t1, t2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s1):
            c = a
            for _ in range(8):
                c = c @ b
            e.record(s1)
            t1.record(s1)
        s2.wait_event(e)
        with torch.cuda.stream(s2):
            t2.record(s2)
            torch.empty(1, device="cuda").zero_()
        torch.cuda.synchronize()
        d.append(t1.elapsed_time(t2) * 1e3)
    d.sort()
    print(f"event timing={timing_evt}: queue-2 marker after queue-1 marker: min {d[0]:.1f} us, "
          f"median {d[len(d) // 2]:.1f} us, max {d[-1]:.1f} us")


if __name__ == "__main__":
    run(False)
    run(True)
