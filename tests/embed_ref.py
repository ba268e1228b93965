"""Torch restatement of the reference embedding server's encode -- the numerics oracle for K7.

LLMEmbeddingModel.encode / mean_pooling (docs/content/docs/en/youtu-embedding/
deploying-locally.mdx:75-79, :81-116), statement for statement: tokenise
(padding, truncation, max_length, special tokens), forward, zero the first
len(tokenizer(instruction)["input_ids"]) mask positions, masked mean in the
hidden dtype promoted to fp32, F.normalize.  Test infrastructure only.
"""
import torch
import torch.nn.functional as Fn


def ref_mean_pooling(hidden_state, attention_mask):
    s = torch.sum(hidden_state * attention_mask.unsqueeze(-1).float(), dim=1)
    d = attention_mask.sum(dim=1, keepdim=True).float()
    return s / d


@torch.no_grad()
def ref_encode(model, tokenizer, sentences, instruction, max_length, device):
    inputs = tokenizer(list(sentences), padding=True, truncation=True, return_tensors="pt", max_length=max_length,
                       add_special_tokens=True)
    inputs = {k: v.to(device) for k, v in inputs.items()}
    last_hidden_state = model(**inputs)[0]
    instruction_tokens = tokenizer(instruction, padding=False, truncation=True, max_length=max_length,
                                   add_special_tokens=True)["input_ids"]
    if len(instruction_tokens) > 0:
        inputs["attention_mask"][:, :len(instruction_tokens)] = 0
    emb = ref_mean_pooling(last_hidden_state, inputs["attention_mask"])
    return Fn.normalize(emb, dim=-1)


def ref_queries(emb, queries):
    return ref_encode(emb.model, emb.tokenizer, [f"{emb.query_instruction}{q}" for q in queries],
                      emb.query_instruction, emb.max_length, emb.device)


def ref_passages(emb, passages):
    return ref_encode(emb.model, emb.tokenizer, [f"{emb.doc_instruction}{p}" for p in passages],
                      emb.doc_instruction, emb.max_length, emb.device)
