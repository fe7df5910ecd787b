"""CPU oracle for the AcinoSet SBA/FTE hot path — TEST INFRASTRUCTURE ONLY.

This package restates the reference's algorithms in float64 numpy so the HIP path
can be checked against it. It is imported only by `tests/`, by
`__graft_entry__.smoke()` (as the checker) and by `bench.py`'s `cpu_baseline`
leg (as the timed CPU port). The product (`acinoset_amd`) never imports it and
has no CPU fallback.

Pinning:
* SBA points-only, projection, triangulation, FK, redescending loss: pinned by the
  golden vectors in tests/golden/ that were produced by running the reference's own
  code (`src/lib/sba.py`, `src/lib/utils.py`, `src/lib/calib.py`, `src/lib/misc.py`,
  `src/lib/metric.py`) in the build container, with a numpy restatement of the four
  OpenCV calls (OpenCV itself is absent: that boundary is *parity unpinned*).
* FTE: **parity unpinned** against IPOPT (Pyomo/IPOPT/HSL are absent, and the
  reference ships no FTE outputs). The oracle restates the objective of
  `src/core/fte.py:435-510` exactly and minimises it with the same safeguarded LM as
  the GPU path; parity is GPU-vs-oracle on identical inputs.
"""
