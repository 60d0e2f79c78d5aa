#!/usr/bin/env python3
"""Extracts the configuration column of the reference's PUSCH decoder vector test table
(tests/unittests/phy/upper/channel_processors/pusch/pusch_decoder_test_data.h:40-217, read as text) into
tests/golden/pusch_decoder_cases.json: per case the segmenter_config fields (codeblock_metadata.h:146-160: base graph,
rv, modulation, Nref, nof_layers, nof_ch_symbols) and the RV sequence. The table's .dat payloads (LLRs and transport
blocks) are absent from the reference snapshot, so tests/test_gpu_hal_cases.py self-generates TBs of a stated size for
each configuration (parity unpinned for the payloads; the configuration space is the reference's). Data only."""
import json
import re
import sys
from pathlib import Path

SRC = Path("/root/reference/tests/unittests/phy/upper/channel_processors/pusch/pusch_decoder_test_data.h")
OUT = Path(__file__).resolve().parent / "pusch_decoder_cases.json"
QM = {"BPSK": 1, "QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}


def main():
    text = SRC.read_text()
    pat = re.compile(r"\{\{ldpc_base_graph_type::BG(\d), (\d+), modulation_scheme::(\w+), (\d+), (\d+), (\d+)\}, "
                     r"\{([\d, ]+)\}, \{\"test_data/pusch_decoder_test_input(\d+)\.dat\"\}")
    cases = []
    for m in pat.finditer(text):
        bg, rv, mod, nref, nl, nsym, rvs, idx = m.groups()
        cases.append({"index": int(idx), "bg": int(bg), "rv": int(rv), "mod": mod, "Qm": QM[mod], "Nref": int(nref),
                      "nof_layers": int(nl), "nof_ch_symbols": int(nsym),
                      "rv_sequence": [int(x) for x in rvs.split(",")]})
    if len(cases) != 174:
        sys.exit(f"expected 174 cases, found {len(cases)}")
    OUT.write_text(json.dumps({"source": "pusch_decoder_test_data.h:40-217", "cases": cases}, indent=0) + "\n")
    print(f"{len(cases)} cases -> {OUT}")


if __name__ == "__main__":
    main()
