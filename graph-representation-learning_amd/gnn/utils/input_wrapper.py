"""Single-vs-batch input handling for predict() (the reference's
handle_single_input / cast_label_to_list, gnn/utils/input_wrapper.py)."""
import inspect
import types
from functools import wraps
from pathlib import Path
from typing import Any

from gnn.utils.json_handler import read_json_file


def _is_single_input(x: Any) -> bool:
    return type(x) not in (list, tuple, types.GeneratorType)


def cast_label_to_list(x: Any) -> Any:
    """A sample given as a JSON path is read; lists/dicts pass through."""
    if isinstance(x, (str, Path)):
        return read_json_file(str(x))
    if isinstance(x, (list, dict)):
        return x
    raise TypeError(f"Unsupported sample type {type(x)}")


def handle_single_input(preprocess_hook=lambda x: x):
    """Apply preprocess_hook to every input; a non-sequence input is wrapped
    into a one-element batch and its result unwrapped again."""

    def decorator(func):
        @wraps(func)
        def wrapped(*args, **kwargs):
            pos = 1 if inspect.getfullargspec(func).args[:1] == ["self"] else 0
            single = _is_single_input(args[pos])
            batch = [args[pos]] if single else args[pos]
            args = list(args)
            args[pos] = [preprocess_hook(x) for x in batch]
            result = func(*args, **kwargs)
            return result[0] if single else result

        return wrapped

    return decorator
