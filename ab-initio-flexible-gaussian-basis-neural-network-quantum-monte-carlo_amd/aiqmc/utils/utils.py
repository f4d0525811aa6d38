"""utils.select_output (AIQMCrelease3/utils/utils.py:1-6)."""
from typing import Any, Callable, Sequence


def select_output(f: Callable[..., Sequence[Any]], argnum: int) -> Callable[..., Any]:
    def f_selected(*args, **kwargs):
        return f(*args, **kwargs)[argnum]
    if hasattr(f, "_aiqmc_network"):
        f_selected._aiqmc_network = f._aiqmc_network
        f_selected._aiqmc_selected = argnum
    return f_selected
