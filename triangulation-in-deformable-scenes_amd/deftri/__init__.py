"""deftri — MI355X-native deformable-triangulation / non-rigid BA solver (hot path of
luicalrob/Triangulation-in-Deformable-Scenes: the g2o LM solve inside arapOptimization).

Layout:
  _abi.py         ctypes mirror of include/deftri.h
  problem.py      flattened graph (numpy) <-> deftri_problem_desc
  mapmodel.py     Map / KeyFrame / MapPoint mirror (the data the solver reads and writes)
  sim.py          synthetic scenes following the reference's simulation path
  capi.py         libdeftri.so binding (HIP kernels behind a C-ABI)
  optimization.py reference-API mirror: arapOptimization, deformationOptimization, ...
  settings.py     Settings YAML subset (the solver's keys)
"""
__all__ = ["_abi", "problem", "mapmodel", "sim", "capi"]
