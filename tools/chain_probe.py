"""Upper bounds for the c3 analysis chain ("Round 6: the c3 step"):
how fast would the pipelined step be if a stage of the chain cost nothing?  Each named
stage runs once (its first call) and every later call returns that first result, so the
step keeps its shape and streams but loses the stage's device (or host) time.  The bench
reuses one slab every step, so the cached results are the ones the stage would compute.
A probe, not a product path: the numbers are bounds on what fusing or removing a stage
could give.

    python tools/chain_probe.py <stages> -- <bench.py arguments>
    stages: comma list of match, vote, merge, lookup, ransac (or "none"); "spin" in
    the list makes the host poll the pipeline's events (hipEventQuery) instead of
    blocking on them (hipEventSynchronize); "hostmaps" makes multidevice.align_split (bench.py
    --single-process) warp every frame behind the host post-processing, as before round 6's
    device-map warp

e.g. python tools/chain_probe.py lookup -- --config c3 --steps 60 --warmup 5 --cpu-sample 0
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _once(fn):
    cache = []

    def wrapped(*a, **k):
        if not cache:
            cache.append(fn(*a, **k))
        return cache[0]
    return wrapped


def main():
    a = sys.argv[1:]
    split = a.index("--") if "--" in a else len(a)
    skip = {s for s in (a[0].split(",") if split > 0 else []) if s and s != "none"}
    unknown = skip - {"match", "vote", "merge", "lookup", "ransac", "spin", "hostmaps"}
    if unknown:
        raise SystemExit(f"chain_probe: unknown stages {sorted(unknown)}")
    import time

    import bench
    from kcmc_amd import pipeline, stages

    if "hostmaps" in skip:  # not a stage: align_split warps behind the host post-processing
        import dataclasses

        from kcmc_amd import distributed as kdist

        kdist.HIP_STAGES = dataclasses.replace(kdist.HIP_STAGES, warp_params=None)
    if "spin" in skip:  # not a stage: the host polls its events instead of blocking on them
        def _wait(self, ev):
            t0 = time.perf_counter()
            while not ev.query():
                pass
            self.stats["wait_s"] += time.perf_counter() - t0
        pipeline.OverlappedSlabs._wait = _wait

    if "match" in skip:
        pipeline.match_stage = _once(pipeline.match_stage)
    if "vote" in skip:
        stages.consensus_vote = _once(stages.consensus_vote)
    if "merge" in skip:  # the merge also writes the consensus pack into the slot's buffer
        choose, first = pipeline.choose_consensus, []

        def choose_once(*args, pack_out=None, **kw):
            if not first:
                first.append((choose(*args, pack_out=pack_out, **kw), None if pack_out is None else pack_out.copy()))
            elif pack_out is not None:
                pack_out[:] = first[0][1]
            return first[0][0]
        pipeline.choose_consensus = choose_once
    if "lookup" in skip:
        pipeline.lookup_stage = _once(pipeline.lookup_stage)
    if "ransac" in skip:
        pipeline.ransac_stage = _once(pipeline.ransac_stage)
    print(f"chain_probe: stages run once: {sorted(skip) or 'none'}", file=sys.stderr, flush=True)
    sys.argv = ["bench.py"] + a[split + 1:]
    bench.main()


if __name__ == "__main__":
    main()
