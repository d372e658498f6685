"""scripts/utils.py of the reference (the parts the evaluation uses): the eval data loader factory
(scripts/utils.py:146-197) lives in lib/data.py; re-exported under the reference's import path."""
from lib.data import make_pairwise_eval_data_loader  # noqa: F401
