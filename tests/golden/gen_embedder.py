"""Golden embeddings from the REFERENCE embedding server's own model code (A4: ``LLMEmbeddingModel`` in
docs/content/docs/en/youtu-embedding/deploying-locally.mdx:41-126: tokenise with right padding and
truncation, transformer forward, zero the attention mask over the instruction's tokens, masked mean-pool,
L2-normalise; query prefix "Instruction: ... \\nQuery:").

Runs only in the build container.  The listing is read from the mdx at run time (its ```python block,
from ``class LLMEmbeddingModel`` up to the server logic) and executed as written on this container's CPU;
nothing of it is copied into the repo.  The model it loads is a small seeded random-init BERT that this
script writes to tests/golden/tiny_bert/ (config, safetensors weights, a WordPiece vocab covering the
texts): no hub download, and the same files load into hiprag's TorchRocmEmbedder on the GPU box.
Output: embedder_golden.json (texts) + embedder_golden.npy (float32 [queries; passages] embeddings).
"""
from __future__ import annotations

import json
import os
import re
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
MDX = "/root/reference/docs/content/docs/en/youtu-embedding/deploying-locally.mdx"
MODEL_DIR = os.path.join(HERE, "tiny_bert")

import numpy as np  # noqa: E402
import torch  # noqa: E402

WORDS = ("course table column grade student teacher schema semester credit campus faculty revenue budget region "
         "quarter invoice order product warehouse shipment retrieve passages answer question search query given "
         "instruction the a of to in for which what how many is are was by with on").split()


def texts():
    rng = np.random.default_rng(21)
    queries = [" ".join(rng.choice(WORDS, int(rng.integers(2, 14)))) + "?" for _ in range(8)]
    passages = [" ".join(rng.choice(WORDS, int(n))) + "." for n in (1, 3, 9, 17, 30, 45, 60, 90, 120, 5, 2, 70)]
    passages.append("Unknown-words: zyx qwv, and " + " ".join(rng.choice(WORDS, 6)))  # [UNK] pieces, punctuation
    return queries, passages


def build_model():
    from transformers import BertConfig, BertModel, BertTokenizer

    os.makedirs(MODEL_DIR, exist_ok=True)
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + list(".,?:-!'\"") + sorted(set(w.lower() for w in WORDS))
    vocab += ["##s", "##ing", "##ed", "un", "##known", "instruction", "query"]
    vocab = list(dict.fromkeys(vocab))
    with open(os.path.join(MODEL_DIR, "vocab.txt"), "w") as f:
        f.write("\n".join(vocab) + "\n")
    BertTokenizer(os.path.join(MODEL_DIR, "vocab.txt"), do_lower_case=True).save_pretrained(MODEL_DIR)
    cfg = BertConfig(vocab_size=len(vocab), hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                     intermediate_size=128, max_position_embeddings=128, hidden_dropout_prob=0.0,
                     attention_probs_dropout_prob=0.0)
    torch.manual_seed(0)
    BertModel(cfg).save_pretrained(MODEL_DIR, safe_serialization=True)


def reference_model_class():
    src = open(MDX, encoding="utf-8").read()
    block = re.search(r"```python\n(.*?)```", src, re.S).group(1)
    head = block[: block.index("class LLMEmbeddingModel")]
    body = block[block.index("class LLMEmbeddingModel"): block.index("# --- Server Logic ---")]
    imports = "\n".join(ln for ln in head.splitlines()
                        if ln.startswith(("from transformers", "from typing", "import torch", "import numpy")))
    ns: dict = {}
    exec(compile(imports + "\n" + body, MDX, "exec"), ns)  # the reference listing, run as written
    return ns["LLMEmbeddingModel"]


def main():
    build_model()
    LLMEmbeddingModel = reference_model_class()
    m = LLMEmbeddingModel(MODEL_DIR, batch_size=128, max_length=64)
    queries, passages = texts()
    q = m.encode_queries(queries).float().cpu().numpy()
    p = m.encode_passages(passages).float().cpu().numpy()
    np.save(os.path.join(HERE, "embedder_golden.npy"), np.concatenate([q, p]).astype(np.float32))
    with open(os.path.join(HERE, "embedder_golden.json"), "w") as f:
        json.dump({"model_dir": "tiny_bert", "max_length": 64, "queries": queries, "passages": passages,
                   "query_instruction": m.query_instruction, "doc_instruction": m.doc_instruction}, f, indent=1)
    print("wrote", q.shape, p.shape, "finite:", bool(np.isfinite(q).all() and np.isfinite(p).all()))


if __name__ == "__main__":
    main()
