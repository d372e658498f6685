"""MI355X-native mirror of the reference's `lib` package (zgojcic/3D_multiview_reg).

Import with `3d_multiview_reg_amd/` on sys.path (as the reference's scripts do
with the repo root):  `import lib.config`, `from lib.utils import ...`.
"""
