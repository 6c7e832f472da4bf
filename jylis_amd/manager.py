"""RepoManagerCore (jylis/repo_manager.pony:36-108): the caller of the hot path.

The reference's actor core does three things the engine depends on:

  converge_deltas(deltas)   `for (k, d) in deltas.values() do _repo.converge(k, d) end`
                            (repo_manager.pony:92-93), one call per decoded peer batch
  flush_deltas(fn)          the heartbeat (cluster.pony:111-134 -> database.pony:42-48):
                            `if _repo.deltas_size() > 0 then fn((_name, _repo.flush_deltas())) end`
                            (repo_manager.pony:86-90)
  _maybe_proactive_flush    after a changing command, at most once per 500 ms
                            (repo_manager.pony:68-84)

This mirror keeps that call sequence unchanged over a GPU repo
(jylis_amd/repo.py), so the per-pair `converge` calls queue and the
heartbeat's `deltas_size()` drains them in one engine call: a replica that
only receives still applies every peer batch within one tick.
"""
import time


class RepoManagerCore:
    def __init__(self, name, repo, clock_ms=None):
        self.name = name
        self.repo = repo
        self._deltas_fn = None
        self._last_proactive = 0
        self._shutdown = False
        self._clock_ms = clock_ms or (lambda: int(time.monotonic() * 1000))

    def converge_deltas(self, deltas):
        """repo_manager.pony:92-93: deltas = [(key, delta)] in array order"""
        for k, d in deltas:
            self.repo.converge(k, d)

    def flush_deltas(self, fn):
        """repo_manager.pony:86-90 (the heartbeat)"""
        self._deltas_fn = fn
        if self.repo.deltas_size() > 0:
            fn((self.name, self.repo.flush_deltas()))

    def changed(self):
        """a command returned `changed` (repo_manager.pony:60-61)"""
        if self._shutdown or self._deltas_fn is None:
            return
        now = self._clock_ms()
        if now - 500 >= self._last_proactive:
            self._deltas_fn((self.name, self.repo.flush_deltas()))
            self._last_proactive = now

    def clean_shutdown(self):
        """repo_manager.pony:95-108: stop accepting requests, flush what is left"""
        self._shutdown = True
        if self._deltas_fn is not None:
            self.flush_deltas(self._deltas_fn)
