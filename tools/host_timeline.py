"""Host-side phase times of the bench step loop (GPU box): wraps Runner.step's calls with
perf_counter and prints per-step means.  python tools/host_timeline.py [bench args...]"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.Counter()


def timed(name, fn):
    def w(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[name] += time.perf_counter() - t
            cnt[name] += 1
    return w


orig_init = bench.Runner.__init__


def init(self, *a, **k):
    orig_init(self, *a, **k)
    c = self.ctx
    for n in ("run_staged", "upload_frames"):
        setattr(c, n, timed(n, getattr(c, n)))
    g = self.gather.g
    if g is not None:
        g.submit = timed("gather.submit", g.submit)
        g.wait = timed("gather.wait", g.wait)
    self.Fr.count_persons = timed("count_persons", self.Fr.count_persons)


bench.Runner.__init__ = init
orig_step = bench.Runner.step
bench.Runner.step = timed("step (total)", orig_step)
sys.argv = ["bench.py", "--no-cpu-baseline", "--no-variants", "--no-profile"] + sys.argv[1:]
bench.main()
for k in sorted(acc, key=lambda k: -acc[k]):
    print("%-16s calls %4d  mean %8.3f ms" % (k, cnt[k], acc[k] / cnt[k] * 1e3), flush=True)
