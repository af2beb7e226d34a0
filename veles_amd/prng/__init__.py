"""Reproducible random number generation (host registry + device kernels)."""
from veles_amd.prng.random_generator import (  # noqa: F401
    RandomGenerator, get, xorshift1024star, xorshift128plus)
