"""DP drivers: same module names as the reference's ``kmerpapa.algorithms`` (v0.2.4).

Only the two lattice-DP modules are on the path; the greedy heuristic,
BayesOpt and all-k-mers models are out of scope.
"""
