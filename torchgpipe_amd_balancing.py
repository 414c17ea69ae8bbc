"""Deprecated module path, kept for parity with ``torchgpipe_balancing``."""
raise ImportError("import 'torchgpipe_amd.balance' instead")
