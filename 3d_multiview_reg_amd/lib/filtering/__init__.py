"""Filtering registry (reference lib/filtering/__init__.py:4-6)."""
from lib.filtering import oanet

filtering_dict = {
    'oanet': oanet.OANet,
}
