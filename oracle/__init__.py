"""CPU oracle (test infrastructure only) -- see stcgan_ref.py."""
