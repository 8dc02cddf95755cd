"""CPU oracle for the NeRF ray-march hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker or the timed CPU baseline.
The product path (``segment-anything-nerf_amd/``) never imports it and fails
loudly when its HIP library is missing.

Contents
  encoders.py  ctypes binding of encoders_oracle.c (C restatement of the
               reference's gridencoder / shencoder / freqencoder .cu kernels)
  renderer.py  torch-CPU restatement of nerf/renderer.py + nerf/network.py
               (+ get_rays from nerf/utils.py), op for op, citing file:line
  tile_codec.py  numpy restatement of the multi-GPU gather's transport record
               (tile_codec.hip), checked against its own error bound
  synth.py     re-export of samnerf_amd/synth.py (deterministic parameter /
               camera synthesis) for the tests and the golden generator

Pinning: tests/test_oracle.py checks this oracle against
  * tests/golden/*.npz -- produced by tools/make_golden.py, which imports the
    reference's own nerf/renderer.py + nerf/network.py in the build container
    (with this C oracle standing in for the CUDA encoders);
  * reference-independent known-answer tests (SciPy spherical harmonics,
    F.grid_sample dense-level trilinear, literal hash vectors).
"""
