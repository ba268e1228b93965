// _hostfast: the store's per-hit result assembly in C (HipVectorStore._assemble, storage.py).  A finished batch of
// B queries x k hits becomes B lists of (Chunk, score) tuples; in Python each hit costs a slotted-dataclass __init__
// frame, two dict lookups and a dict copy (~2 us), which bounds the store's event loop at ~23k queries/s while the
// GPU serves 52k.  Here each Chunk is allocated with its type's tp_alloc and its six slots are written at the member
// offsets read from the class once (no __init__ frame: the dataclass __init__ only assigns the fields), with the same
// values the Python loop produces: id = rec[0], document_id = meta.get("document_id", ""), content = rec[2],
// chunk_index = meta.get("chunk_index", 0), metadata = a fresh copy of meta, embedding = embs[j] or None.
// A batch's hits would be 2 tracked objects each (the Chunk and its pair tuple): walked by every gen-0 pass of the
// cycle collector and promoted with the results held, the collector cost more than the assembly did
// (tools/bench_store_host.py); the caller may therefore ask for atomic-valued hits to be left untracked (see below,
// off by default).  The collector itself is never switched off.
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

static const char* kFields[6] = {"id", "document_id", "content", "chunk_index", "metadata", "embedding"};
static const char* kResultFields[3] = {"chunk", "score", "rank"};

static int slot_offsets_of(PyTypeObject* cls, const char* const* fields, int n, Py_ssize_t* off) {
    for (int f = 0; f < n; ++f) {
        PyObject* d = PyObject_GetAttrString((PyObject*)cls, fields[f]);  // the class attribute: a member descriptor
        if (!d) return -1;
        if (!PyObject_TypeCheck(d, &PyMemberDescr_Type) || ((PyMemberDescrObject*)d)->d_member->type != T_OBJECT_EX) {
            Py_DECREF(d);
            PyErr_Format(PyExc_TypeError, "%s.%s is not a __slots__ member", cls->tp_name, fields[f]);
            return -1;
        }
        off[f] = ((PyMemberDescrObject*)d)->d_member->offset;
        Py_DECREF(d);
    }
    return 0;
}

static int slot_offsets(PyTypeObject* cls, Py_ssize_t off[6]) { return slot_offsets_of(cls, kFields, 6, off); }

// one hit's Chunk (a new reference): the fields as assemble writes them (see the header)
static PyObject* make_chunk(PyTypeObject* cls, const Py_ssize_t off[6], PyObject* r, PyObject* m, PyObject* emb,
                            PyObject* k_doc, PyObject* k_idx, PyObject* empty, PyObject* zero) {
    if (!PyTuple_Check(r) || PyTuple_GET_SIZE(r) < 3 || !PyDict_Check(m)) {
        PyErr_SetString(PyExc_TypeError, "a host record is not (id, _, content) with a metadata dict");
        return NULL;
    }
    PyObject* doc = PyDict_GetItemWithError(m, k_doc);
    if (!doc && PyErr_Occurred()) return NULL;
    PyObject* idx = PyDict_GetItemWithError(m, k_idx);
    if (!idx && PyErr_Occurred()) return NULL;
    PyObject* md = PyDict_Copy(m);
    if (!md) return NULL;
    PyObject* c = cls->tp_alloc(cls, 0);
    if (!c) {
        Py_DECREF(md);
        return NULL;
    }
    PyObject* vals[6] = {PyTuple_GET_ITEM(r, 0), doc ? doc : empty, PyTuple_GET_ITEM(r, 2), idx ? idx : zero, md, emb};
    for (int f = 0; f < 6; ++f) {
        if (f != 4) Py_INCREF(vals[f]);  // (md: the new reference moves in)
        *(PyObject**)((char*)c + off[f]) = vals[f];
    }
    return c;
}

// assemble(cls, rec_l, meta_l, score_l, per_q, embs, untrack=0) -> list of B lists of (cls instance, float)
static PyObject* assemble(PyObject* self, PyObject* args) {
    PyTypeObject* cls;
    PyObject *recs, *metas, *scores, *per_q, *embs;
    int untrack = 0;
    if (!PyArg_ParseTuple(args, "O!O!O!O!O!O|p", &PyType_Type, &cls, &PyList_Type, &recs, &PyList_Type, &metas,
                          &PyList_Type, &scores, &PyList_Type, &per_q, &embs, &untrack))
        return NULL;
    if (cls->tp_dictoffset != 0) return PyErr_Format(PyExc_TypeError, "%s has a __dict__", cls->tp_name);
    Py_ssize_t off[6];
    if (slot_offsets(cls, off)) return NULL;
    const Py_ssize_t n_hits = PyList_GET_SIZE(recs);
    if (PyList_GET_SIZE(metas) != n_hits || PyList_GET_SIZE(scores) != n_hits ||
        (embs != Py_None && (!PyList_Check(embs) || PyList_GET_SIZE(embs) != n_hits)))
        return PyErr_Format(PyExc_ValueError, "hit lists of different lengths");
    PyObject* k_doc = PyUnicode_InternFromString("document_id");
    PyObject* k_idx = PyUnicode_InternFromString("chunk_index");
    PyObject* empty = PyUnicode_FromString("");
    PyObject* zero = PyLong_FromLong(0);
    const Py_ssize_t B = PyList_GET_SIZE(per_q);
    PyObject* out = PyList_New(B);
    if (!k_doc || !k_idx || !empty || !zero || !out) goto fail;
    Py_ssize_t j = 0;
    for (Py_ssize_t q = 0; q < B; ++q) {
        const Py_ssize_t cnt = PyLong_AsSsize_t(PyList_GET_ITEM(per_q, q));
        if (cnt < 0 || j + cnt > n_hits) {
            if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "per-query counts exceed the hits");
            goto fail;
        }
        PyObject* res = PyList_New(0);
        if (!res) goto fail;
        PyList_SET_ITEM(out, q, res);
        for (Py_ssize_t e = j + cnt; j < e; ++j) {
            PyObject* r = PyList_GET_ITEM(recs, j);
            if (r == Py_None) continue;  // a row deleted since the search ran
            PyObject* m = PyList_GET_ITEM(metas, j);
            PyObject* emb = embs == Py_None ? Py_None : PyList_GET_ITEM(embs, j);
            PyObject* c = make_chunk(cls, off, r, m, emb, k_doc, k_idx, empty, zero);
            if (!c) goto fail;
            PyObject* md = *(PyObject**)((char*)c + off[4]);
            PyObject* pair = PyTuple_New(2);
            if (!pair) {
                Py_DECREF(c);
                goto fail;
            }
            PyObject* s = PyList_GET_ITEM(scores, j);
            Py_INCREF(s);
            PyTuple_SET_ITEM(pair, 0, c);
            PyTuple_SET_ITEM(pair, 1, s);
            if (untrack && !PyObject_GC_IsTracked(md) && (emb == Py_None || !PyObject_IS_GC(emb))) {
                // (opt-in: index_params.untracked_results) a Chunk of strings, numbers and an untracked
                // (atomic-valued) metadata dict references no container that can lead back to it, so the cycle
                // collector is given none of a batch's hits to walk, as CPython does for tuples and dicts of atomic
                // values.  What this gives up: a slotted instance is not re-tracked when a container is stored in
                // it later, so a cycle a caller builds THROUGH a returned Chunk (its own metadata holding the
                // Chunk) is never collected -- hence off by default.
                PyObject_GC_UnTrack(c);
                PyObject_GC_UnTrack(pair);
            }
            if (PyList_Append(res, pair)) {
                Py_DECREF(pair);
                goto fail;
            }
            Py_DECREF(pair);
        }
    }
    Py_DECREF(k_doc);
    Py_DECREF(k_idx);
    Py_DECREF(empty);
    Py_DECREF(zero);
    return out;
fail:
    Py_XDECREF(k_doc);
    Py_XDECREF(k_idx);
    Py_XDECREF(empty);
    Py_XDECREF(zero);
    Py_XDECREF(out);
    return NULL;
}

// assemble_results(chunk_cls, result_cls, rec_l, meta_l, score_l, per_q, embs, top_k_l, threshold_l, untrack=0) ->
// list of B lists of result_cls(chunk, score, rank): what VectorRetriever's _to_results makes of assemble's pairs for
// a call with that top_k and similarity threshold (base_retriever.py:66-80 without a reranker) -- the first top_k
// live hits, rank = position + 1 among them BEFORE the threshold drops any (a threshold <= 0 keeps all) -- without
// the intermediate (Chunk, score) tuple, and without building the Chunks of hits past a call's own top_k.
static PyObject* assemble_results(PyObject* self, PyObject* args) {
    PyTypeObject *cls, *rcls;
    PyObject *recs, *metas, *scores, *per_q, *embs, *ks, *ths;
    int untrack = 0;
    if (!PyArg_ParseTuple(args, "O!O!O!O!O!O!OO!O!|p", &PyType_Type, &cls, &PyType_Type, &rcls, &PyList_Type, &recs,
                          &PyList_Type, &metas, &PyList_Type, &scores, &PyList_Type, &per_q, &embs, &PyList_Type, &ks,
                          &PyList_Type, &ths, &untrack))
        return NULL;
    if (cls->tp_dictoffset != 0 || rcls->tp_dictoffset != 0)
        return PyErr_Format(PyExc_TypeError, "%s / %s has a __dict__", cls->tp_name, rcls->tp_name);
    Py_ssize_t off[6], roff[3];
    if (slot_offsets(cls, off) || slot_offsets_of(rcls, kResultFields, 3, roff)) return NULL;
    const Py_ssize_t n_hits = PyList_GET_SIZE(recs);
    const Py_ssize_t B = PyList_GET_SIZE(per_q);
    if (PyList_GET_SIZE(metas) != n_hits || PyList_GET_SIZE(scores) != n_hits ||
        (embs != Py_None && (!PyList_Check(embs) || PyList_GET_SIZE(embs) != n_hits)) || PyList_GET_SIZE(ks) != B ||
        PyList_GET_SIZE(ths) != B)
        return PyErr_Format(PyExc_ValueError, "hit / query lists of different lengths");
    PyObject* k_doc = PyUnicode_InternFromString("document_id");
    PyObject* k_idx = PyUnicode_InternFromString("chunk_index");
    PyObject* empty = PyUnicode_FromString("");
    PyObject* zero = PyLong_FromLong(0);
    PyObject* out = PyList_New(B);
    if (!k_doc || !k_idx || !empty || !zero || !out) goto fail;
    Py_ssize_t j = 0;
    for (Py_ssize_t q = 0; q < B; ++q) {
        const Py_ssize_t cnt = PyLong_AsSsize_t(PyList_GET_ITEM(per_q, q));
        const Py_ssize_t kq = PyLong_AsSsize_t(PyList_GET_ITEM(ks, q));
        const double th = PyFloat_AsDouble(PyList_GET_ITEM(ths, q));
        if (PyErr_Occurred()) goto fail;
        if (cnt < 0 || j + cnt > n_hits) {
            PyErr_SetString(PyExc_ValueError, "per-query counts exceed the hits");
            goto fail;
        }
        PyObject* res = PyList_New(0);
        if (!res) goto fail;
        PyList_SET_ITEM(out, q, res);
        Py_ssize_t pos = 0;  // live hits of this query so far (the rank before the threshold)
        for (Py_ssize_t e = j + cnt; j < e; ++j) {
            PyObject* r = PyList_GET_ITEM(recs, j);
            if (r == Py_None) continue;  // a row deleted since the search ran
            if (pos >= kq) continue;
            ++pos;
            PyObject* s = PyList_GET_ITEM(scores, j);
            const double sv = PyFloat_AsDouble(s);
            if (sv == -1.0 && PyErr_Occurred()) goto fail;
            if (th > 0.0 && !(sv >= th)) continue;
            PyObject* emb = embs == Py_None ? Py_None : PyList_GET_ITEM(embs, j);
            PyObject* c = make_chunk(cls, off, r, PyList_GET_ITEM(metas, j), emb, k_doc, k_idx, empty, zero);
            if (!c) goto fail;
            PyObject* rank = PyLong_FromSsize_t(pos);
            PyObject* rr = rank ? rcls->tp_alloc(rcls, 0) : NULL;
            if (!rr) {
                Py_XDECREF(rank);
                Py_DECREF(c);
                goto fail;
            }
            Py_INCREF(s);
            *(PyObject**)((char*)rr + roff[0]) = c;
            *(PyObject**)((char*)rr + roff[1]) = s;
            *(PyObject**)((char*)rr + roff[2]) = rank;
            PyObject* md = *(PyObject**)((char*)c + off[4]);
            if (untrack && !PyObject_GC_IsTracked(md) && (emb == Py_None || !PyObject_IS_GC(emb))) {
                PyObject_GC_UnTrack(c);  // (opt-in, as in assemble; the result then holds only untracked objects)
                PyObject_GC_UnTrack(rr);
            }
            if (PyList_Append(res, rr)) {
                Py_DECREF(rr);
                goto fail;
            }
            Py_DECREF(rr);
        }
    }
    Py_DECREF(k_doc);
    Py_DECREF(k_idx);
    Py_DECREF(empty);
    Py_DECREF(zero);
    return out;
fail:
    Py_XDECREF(k_doc);
    Py_XDECREF(k_idx);
    Py_XDECREF(empty);
    Py_XDECREF(zero);
    Py_XDECREF(out);
    return NULL;
}

static PyMethodDef kMethods[] = {
    {"assemble", assemble, METH_VARARGS, "assemble(cls, rec_l, meta_l, score_l, per_q, embs, untrack=False) -> list[list[(cls, score)]]"},
    {"assemble_results", assemble_results, METH_VARARGS,
     "assemble_results(chunk_cls, result_cls, rec_l, meta_l, score_l, per_q, embs, top_k_l, threshold_l, untrack=False) -> "
     "list[list[result_cls]]"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_hostfast", NULL, -1, kMethods};

PyMODINIT_FUNC PyInit__hostfast(void) { return PyModule_Create(&kModule); }
