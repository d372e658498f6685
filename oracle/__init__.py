"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A numpy restatement of the reference (zgojcic/3D_multiview_reg) pairwise
registration hot path, used *only* as the checker by tests/, by
`__graft_entry__.smoke()` and as the `cpu_baseline` leg of bench.py.  The
product path (3d_multiview_reg_amd/) never imports this package and fails
loudly if its HIP library is missing.

Pinning: kabsch / oanet / soft_nn / sampler / pairs are checked against golden
vectors produced by running the reference's own code in the build container
(tests/golden/make_golden.py -> tests/golden/*.npz; tests/test_oracle_golden.py).
The FCGF sparse-conv restatement (oracle/fcgf.py) and FPS (oracle/fps.py)
restate un-vendored third-party libraries (MinkowskiEngine 0.4.x,
pointnet2_ops) that cannot run here: "parity unpinned" for those two
(DESIGN.md §Oracle).
"""
