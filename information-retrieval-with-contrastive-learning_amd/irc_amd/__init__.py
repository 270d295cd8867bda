"""irc_amd -- MI355X-native (gfx950) kernels + host runtime for the contrastive
training and dense retrieval hot path of PM25/Information-Retrieval-with-
Contrastive-Learning.  See DESIGN.md at the repository root."""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
