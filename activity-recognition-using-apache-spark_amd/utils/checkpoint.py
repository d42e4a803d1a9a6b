"""Training checkpoints, resume and fault injection (the reference has
no checkpointing; Spark only re-computes lost partitions from lineage).

* ``Checkpointer(dir)`` writes ``ckpt-<step>.pt`` atomically (temp file + rename)
  holding tensors only (``torch.load(weights_only=True)``-safe) plus a small JSON
  sidecar; ``latest()`` finds the newest complete checkpoint, so a job restarted by
  ``torchrun --max-restarts`` (or by hand) resumes where it stopped.
* MLP training checkpoints (parameters, Adam moments, step counter, epoch/step,
  data-order RNG state) every ``every`` steps; RandomForest checkpoints after
  each completed wave of trees.
* Every checkpoint records a ``fingerprint`` of the fit that wrote it (model
  hyper-parameters, data shape, world size); ``latest(fingerprint=...)`` ignores a
  checkpoint whose fingerprint differs, so a stale directory never resumes a
  different configuration.
* Fault injection for tests: ``HAR_FAULT_INJECT="<step>"`` or ``"<rank>:<step>"``
  makes ``maybe_inject_fault`` hard-exit the process (exit code 17) when training
  reaches that step — exactly like a crashed rank.  Under ``torchrun --max-restarts`` the fault
  fires on the first attempt only (``TORCHELASTIC_RESTART_COUNT`` = 0): the restarted group resumes
  from the newest checkpoint and runs to the end (``tests/test_checkpoint.py``).
"""
from __future__ import annotations

import glob
import json
import os
import re
import warnings
from typing import Dict, Optional

import torch

FAULT_EXIT_CODE = 17


class Checkpointer:
    def __init__(self, directory: str, keep: int = 2, rank: int = 0):
        self.dir = directory
        self.keep = keep
        self.rank = rank
        os.makedirs(directory, exist_ok=True)

    def save(self, step: int, tensors: Dict[str, torch.Tensor], meta: Optional[dict] = None,
             fingerprint: Optional[dict] = None):
        if self.rank != 0:  # replicated state: one writer
            return
        meta = dict(meta or {})
        if fingerprint is not None:
            meta["fingerprint"] = _canon(fingerprint)
        path = os.path.join(self.dir, f"ckpt-{step:09d}.pt")
        tmp = path + ".tmp"
        torch.save({k: v.detach().cpu() if isinstance(v, torch.Tensor) else torch.as_tensor(v)
                    for k, v in tensors.items()}, tmp)
        with open(path + ".json.tmp", "w") as f:
            json.dump({"step": step, **(meta or {})}, f)
        os.replace(tmp, path)
        os.replace(path + ".json.tmp", path + ".json")
        for old in self._all()[:-self.keep]:
            for p in (old, old + ".json"):
                if os.path.exists(p):
                    os.remove(p)

    def _all(self):
        files = [p for p in glob.glob(os.path.join(self.dir, "ckpt-*.pt")) if os.path.exists(p + ".json")]
        return sorted(files, key=lambda p: int(re.findall(r"ckpt-(\d+)\.pt", p)[0]))

    def latest(self, fingerprint: Optional[dict] = None):
        """Newest complete checkpoint as ``(tensors, meta)``; with ``fingerprint``, None when the
        newest checkpoint was written by a fit with other parameters or data."""
        files = self._all()
        if not files:
            return None
        p = files[-1]
        with open(p + ".json") as f:
            meta = json.load(f)
        if fingerprint is not None and meta.get("fingerprint") != _canon(fingerprint):
            warnings.warn(f"ignoring checkpoint {p}: written by a different fit "
                          f"({meta.get('fingerprint')} != {_canon(fingerprint)})")
            return None
        return torch.load(p, weights_only=True, map_location="cpu"), meta


def _canon(d: dict) -> dict:
    """JSON-stable form of a fingerprint (tuples -> lists, numpy scalars -> python)."""
    return json.loads(json.dumps(d, sort_keys=True, default=lambda o: o.item() if hasattr(o, "item") else str(o)))


def maybe_inject_fault(step: int, rank: int = 0):
    spec = os.environ.get("HAR_FAULT_INJECT", "")
    if not spec or int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")) > 0:
        return
    if ":" in spec:
        r, s = spec.split(":", 1)
        if int(r) != rank:
            return
    else:
        s = spec
    if int(s) == step:
        import sys

        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(FAULT_EXIT_CODE)
