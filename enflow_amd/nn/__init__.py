from .egcl import EGCL  # noqa: F401
from .argmax import ArgMax  # noqa: F401
from .floor import Floor  # noqa: F401
