"""Descriptor registry (reference lib/descriptor/__init__.py:3-5)."""
from lib.descriptor import fcgf

descriptor_dict = {
    'fcgf': fcgf.FCGFNet,
}
