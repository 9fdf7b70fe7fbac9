"""Text-table readers of the espnet2 data directory (espnet2/fileio/read_text.py:5-65).

`read_2column_text`: "key value..." per line -> {key: value} (value = rest of the line; a
key alone maps to ""); a repeated key raises RuntimeError (read_text.py:17-25).
`load_num_sequence_text`: "key n1<delim>n2..." -> {key: [numbers]} with the delimiter and
number type chosen by loader_type (text_int / text_float: space, csv_int / csv_float: comma;
read_text.py:38-63).  Both are host-side bookkeeping for the data feed.
"""
from pathlib import Path
from typing import Dict, List, Union

_NUM_LOADERS = {"text_int": (" ", int), "text_float": (" ", float), "csv_int": (",", int),
                "csv_float": (",", float)}


def read_2column_text(path: Union[Path, str]) -> Dict[str, str]:
    table: Dict[str, str] = {}
    with Path(path).open("r", encoding="utf-8") as f:
        for lineno, raw in enumerate(f, 1):
            parts = raw.rstrip().split(maxsplit=1)
            key = parts[0] if parts else ""
            val = parts[1] if len(parts) > 1 else ""
            if key in table:
                raise RuntimeError(f"{key} is duplicated ({path}:{lineno})")
            table[key] = val
    return table


def load_num_sequence_text(path: Union[Path, str], loader_type: str = "csv_int") -> Dict[str, List]:
    if loader_type not in _NUM_LOADERS:
        raise ValueError(f"Not supported loader_type={loader_type}")
    delim, conv = _NUM_LOADERS[loader_type]
    out = {}
    for key, val in read_2column_text(path).items():
        try:
            out[key] = [conv(tok) for tok in val.split(delim)]
        except (TypeError, ValueError):
            raise ValueError(f"Error happened with path={path}, id={key}, value={val}") from None
    return out
