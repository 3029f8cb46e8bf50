"""Wall-clock stack sampler for the host side of a run: a daemon thread snapshots the main
thread's Python stack every `interval` seconds (sys._current_frames) and counts, per sample,
the innermost frames and the innermost repository frame.  Unlike cProfile it adds no per-call
overhead and attributes device waits (a blocking .to('cpu') / .item()) to the code that waits.

    from tools.stack_sampler import Sampler
    with Sampler() as s: ...;  s.report(path)
"""
import collections
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class Sampler:
    def __init__(self, interval=0.0005, thread_id=None):
        self.interval = interval
        self.tid = thread_id or threading.get_ident()
        self.leaf = collections.Counter()
        self.repo = collections.Counter()
        self.stacks = collections.Counter()
        self.n = 0
        self._stop = threading.Event()
        self._t = None

    def _run(self):
        while not self._stop.is_set():
            f = sys._current_frames().get(self.tid)
            if f is not None:
                self.n += 1
                self.leaf[f"{f.f_code.co_filename.replace(REPO + '/', '')}:{f.f_lineno} {f.f_code.co_name}"] += 1
                chain = []
                g = f
                while g is not None and len(chain) < 6:
                    fn = g.f_code.co_filename
                    if fn.startswith(REPO):
                        chain.append(f"{fn.replace(REPO + '/', '')}:{g.f_lineno} {g.f_code.co_name}")
                    g = g.f_back
                if chain:
                    self.repo[chain[0]] += 1
                    self.stacks[" <- ".join(chain[:4])] += 1
            time.sleep(self.interval)

    def __enter__(self):
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join()

    def report(self, path, top=40):
        lines = [f"samples: {self.n} (interval {self.interval * 1e3:.2f} ms)", "", "innermost frame:"]
        for k, v in self.leaf.most_common(top):
            lines.append(f"  {100.0 * v / max(self.n, 1):6.2f}%  {k}")
        lines += ["", "innermost repository frame:"]
        for k, v in self.repo.most_common(top):
            lines.append(f"  {100.0 * v / max(self.n, 1):6.2f}%  {k}")
        lines += ["", "repository stacks (4 deep):"]
        for k, v in self.stacks.most_common(top):
            lines.append(f"  {100.0 * v / max(self.n, 1):6.2f}%  {k}")
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
