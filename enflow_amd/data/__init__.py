from .base import Data, Edges, DataLoader  # noqa: F401
