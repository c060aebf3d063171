"""ORACLE — test infrastructure, never the product.

A CPU restatement of the reference's AC/TC scoring path (XThomasBU/video-gen-evals), used only as
the checker: by ``tests/``, by ``__graft_entry__.smoke()`` and by ``bench.py``'s ``cpu_baseline``
leg.  The product (``video-gen-evals_amd/vge`` + ``libvge.so``) never imports anything here and
fails loudly when its HIP library is missing.

Modules (each function cites the reference file:line it restates):
  lapack2x2  -- LAPACK sgesdd on 2x2 matrices (the sign convention utils.py:207-212 depends on)
  featurize  -- utils.py:130-217 (deltas), 366-516 (window featurisation), 589-801 (stats)
  encoder    -- model.py:8-193 (HumanActionScorer forward) as torch-fp32 functional code
  evalflow   -- eval.py:48-466 + utils.py:326-341, 803-911, 1018-1045 (the scoring driver)

Parity of the oracle itself is pinned by tests/test_oracle_golden.py against golden vectors that
tests/golden/make_golden.py produced by importing the reference in the build container.
"""
