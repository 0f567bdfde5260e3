"""CPU oracle for the CC-MPC Monte-Carlo prediction + MVOE chance-constraint path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (``cc-mpc_amd/ccmpc``) imports,
links or executes anything under ``oracle/``.  Only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` may use it, and only as the checker / the timed
CPU baseline -- never as the thing measured or shipped.

Contents
  ccmpc_oracle.py  NumPy restatement of the reference's algorithm, loop-faithful, each function
                   citing the reference file:line it follows.
  philox.py        The counter RNG the HIP kernels use, so injected randomness is reproducible.

Pinning: the math kernels (compute_mvoe, predict_moments, choose_closest_tangent,
compute_lower_bound, compute_scale) are checked against golden vectors produced by the
reference's own ``makeconstraint.py`` (``tests/golden/make_golden.py``).  The planner glue
(v8ideal/__init__.py) cannot be imported here (it needs carla, cvxpy, docplex, control and
Trajectron++, none installed), so its golden cycles are produced by the restated glue driving
the reference's makeconstraint functions.  The Trajectron++ sampler restatement is
"parity unpinned" (the submodule is absent, no reference test pins it).
"""
