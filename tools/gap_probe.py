"""Probe of the idle time between a warp and the next slab's knn2 in the pipelined c2 step
("Kernel boundaries").  Run under a kernel trace, one variant per run:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap/<v> -o run -- \
        python tools/gap_probe.py <variant> [--steps 12]
    python tools/gap_probe.py --report gpurun_out/gap

variants: base (OverlappedSlabs as shipped), nowait (no check of the caller's stream per
submit), notiming (the kernel-stream tail events without timing), both, squery (the
caller's stream asked with hipStreamQuery instead of an event recorded on it), onstream
(the caller on a stream of its own instead of the null stream), lazytail (no event
between the warp and the next match), tiny (a small elementwise kernel before each
match: is the idle time the warp's or the knn2's?), nocorun (RANSAC behind the warp on
the kernel stream: nothing runs beside the warp)."""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def report(root):
    import numpy as np

    for d in sorted(glob.glob(os.path.join(root, "*"))):
        rows = []
        for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(p) as f:
                for r in csv.DictReader(f):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]))
        rows.sort()
        gaps, first = [], []
        warp_end = prev_end = None
        warp_q = None
        for s, e, n, q in rows:
            if "warp_affine_u16_kernel" in n:
                warp_end, warp_q = e, q
                first.append(None)
            elif warp_end is not None and first and first[-1] is None and q == warp_q:
                first[-1] = (n.replace("void ", "").replace("(anonymous namespace)::", "")[:28], (s - warp_end) / 1e3)
            if "knn2_l2u8_kernel" in n and warp_end is not None:
                gaps.append(((s - warp_end) / 1e3, (s - prev_end) / 1e3))
                warp_end = None
            if "ransac" not in n and "copyBuffer" not in n:
                prev_end = e
        g = np.array(gaps[2:]) if len(gaps) > 3 else np.array(gaps)
        if g.size:
            print(f"{os.path.basename(d):10s} warp end -> knn2 start: median {np.median(g[:, 0]):6.1f} us, "
                  f"min {g[:, 0].min():6.1f}, max {g[:, 0].max():6.1f} (n={len(g)}); "
                  f"idle right before knn2 {np.median(g[:, 1]):6.1f} us")
            fk = [x for x in first[2:] if x is not None]
            if fk:
                print(f"{'':10s} first kernel after the warp: {fk[0][0]}, median {np.median([x[1] for x in fk]):6.1f} us")


def main():
    a = sys.argv[1:]
    if a and a[0] == "--report":
        return report(a[1])
    variant = a[0] if a else "base"
    steps = int(a[a.index("--steps") + 1]) if "--steps" in a else 12
    import torch

    import bench
    from kcmc_amd import pipeline

    if variant in ("nowait", "both"):
        pipeline.OverlappedSlabs._wait_current = lambda self: None
    if variant == "squery":  # ask the caller's stream itself whether work is pending
        def _wait_current(self):
            cur = torch.cuda.current_stream(self.dev)
            if cur == self.stream or cur.query():
                return
            ev = torch.cuda.Event()
            ev.record(cur)
            self.stream.wait_event(ev)
            self._queued()
        pipeline.OverlappedSlabs._wait_current = _wait_current
    if variant == "onstream":  # the caller runs on a stream of its own (not the null stream)
        side = torch.cuda.Stream()
    if variant == "lazytail":  # an event at the kernel stream's tail only behind the match
        def _at_tail(self, mark, *names):
            if "m1" not in names:
                return torch.cuda.Event()  # never recorded: waits and queries on it pass
            if self._tail is None:
                self._tail = torch.cuda.Event()
                self._tail.record(self.stream)
            return self._tail
        pipeline.OverlappedSlabs._at_tail = _at_tail
    if variant == "tiny":  # a tiny elementwise kernel right before every match
        tiny = torch.zeros(64, device="cuda")
        match_stage = pipeline.match_stage

        def _match_stage(inp, cfg):
            tiny.add_(1)
            return match_stage(inp, cfg)
        pipeline.match_stage = _match_stage
    if variant in ("notiming", "both"):
        def _at_tail(self, mark, *names):
            if self._tail is None:
                self._tail = torch.cuda.Event()
                self._tail.record(self.stream)
            return self._tail
        pipeline.OverlappedSlabs._at_tail = _at_tail
    bc = bench.CONFIGS["c2"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    inp, _ = bench.make_inputs(bc, bc.frames_per_gpu, 0, dev)
    out = torch.empty_like(inp.frames)
    cfg = pipeline.AlignConfig(n_kp_global=bc.n_kp_global, ransac_model=bc.model)
    ov = pipeline.OverlappedSlabs(dev, cfg)
    torch.cuda.synchronize()
    with torch.cuda.stream(side if variant == "onstream" else torch.cuda.current_stream()):
        for _ in range(steps):
            ov.submit(inp, out=out)
        ov.flush()
    ov.synchronize()
    print(f"{variant}: {steps} steps done")


if __name__ == "__main__":
    main()
