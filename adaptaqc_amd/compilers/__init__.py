from .adapt.adapt_compiler import AdaptCompiler  # noqa: F401
from .adapt.adapt_config import AdaptConfig  # noqa: F401
from .adapt.adapt_result import AdaptResult  # noqa: F401
from .approximate_compiler import ApproximateCompiler  # noqa: F401
