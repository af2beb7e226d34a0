"""Run reports (reference veles/publishing/)."""
from veles_amd.publishing.publisher import Publisher  # noqa: F401
