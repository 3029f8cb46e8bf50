"""Metadata (.mtd) JSON files next to data files (reference: parser/DataExpression.java
readMetadataFile / runtime/util/MapReduceTool.writeMetaDataFile)."""
from __future__ import annotations

import json
import os


def mtd_path(fname):
    return fname + ".mtd"


def read_mtd(fname):
    p = mtd_path(fname)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        txt = f.read()
    try:
        return json.loads(txt)
    except json.JSONDecodeError:
        # tolerate the reference's lenient JSON (unquoted keys / trailing commas)
        import re
        t = re.sub(r"([{,]\s*)([A-Za-z_][A-Za-z0-9_]*)\s*:", r'\1"\2":', txt)
        t = re.sub(r",\s*}", "}", t)
        return json.loads(t)


def write_mtd(fname, data_type, value_type, rows, cols, nnz=None, fmt="text", schema=None, **extra):
    md = {"data_type": data_type, "value_type": value_type, "rows": int(rows), "cols": int(cols)}
    if nnz is not None:
        md["nnz"] = int(nnz)
    md["format"] = fmt
    if schema is not None:
        md["schema"] = schema
    md.update(extra)
    md["author"] = "systemml_amd"
    with open(mtd_path(fname), "w") as f:
        json.dump(md, f, indent=4)
