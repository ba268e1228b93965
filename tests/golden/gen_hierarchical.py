"""Golden outputs of the REFERENCE's HierarchicalMarkdownSplitter (utu/rag/knowledge_builder/chunker.py:124-349),
the splitter processors.py:371-379 uses for ``*_chunklevel.md`` documents.  Runs only in the build
container (reference tree read-only, no bytecode written); the module imports without stand-ins.
Inputs: seeded synthetic markdown (H1 / H2 / H3 lines, blank lines, lines longer than a chunk, headers
made of spaces, '#' without a space, text before the first header, CRLF line ends) under four chunk
configs.  Output: hierarchical.json (inputs and the splitter's chunks)."""
from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from gen_golden import load_reference  # noqa: E402

WORDS = ("course table column grade student teacher schema semester credit campus faculty revenue budget region "
         "quarter invoice order product warehouse").split()


def markdown(rng) -> str:
    lines = []
    if rng.random() < 0.5:
        lines.append("preamble " + " ".join(rng.choice(WORDS, int(rng.integers(3, 12)))))
    for _ in range(int(rng.integers(1, 5))):
        kind = rng.random()
        if kind < 0.1:
            lines.append("#   ")  # a header of spaces: truthiness of its stripped text
        elif kind < 0.15:
            lines.append("#no-space heading is content")
        else:
            lines.append("# " + " ".join(rng.choice(WORDS, int(rng.integers(1, 4)))).title() + "  ")
        for _ in range(int(rng.integers(0, 4))):
            if rng.random() < 0.8:
                lines.append("## " + " ".join(rng.choice(WORDS, int(rng.integers(1, 4)))))
            for _ in range(int(rng.integers(0, 7))):
                r = rng.random()
                if r < 0.15:
                    lines.append("")
                elif r < 0.2:
                    lines.append("   ")
                elif r < 0.27:
                    lines.append("### " + " ".join(rng.choice(WORDS, 3)))
                elif r < 0.32:
                    lines.append(" ".join(rng.choice(WORDS, int(rng.integers(40, 90)))))  # longer than a chunk
                else:
                    lines.append(("  " if rng.random() < 0.2 else "") + " ".join(rng.choice(WORDS, int(rng.integers(2, 20)))))
    text = "\n".join(lines)
    if rng.random() < 0.15:
        text = text.replace("\n", "\r\n")
    return text


def main():
    mods = load_reference()
    chunker, config = mods["chunker"], mods["config"]
    rng = np.random.default_rng(11)
    texts = [markdown(rng) for _ in range(40)] + ["", "   \n\n ", "# Only A Header", "## only h2\nbody line",
                                                 "plain text\nwithout headers\n\nat all"]
    cfgs = [(100, 0), (200, 30), (500, 50), (1000, 100), (150, 1000)]
    cases = []
    for size, ov in cfgs:
        sp = chunker.HierarchicalMarkdownSplitter(config.ChunkingConfig(strategy="hierarchical", chunk_size=size,
                                                                         chunk_overlap=ov))
        cases.append({"chunk_size": size, "chunk_overlap": ov, "chunks": [sp.split_text(t) for t in texts]})
    with open(os.path.join(HERE, "hierarchical.json"), "w") as f:
        json.dump({"texts": texts, "cases": cases}, f, indent=0, ensure_ascii=False)
    print("wrote", os.path.join(HERE, "hierarchical.json"), sum(len(c) for k in cases for c in k["chunks"]), "chunks")


if __name__ == "__main__":
    main()
