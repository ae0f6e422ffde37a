/* CPython binding of the library's per-call host entry K8a (avdb_annotate_host)
 * for the drop-in VariantAnnotator (Util/lib/python/variant_annotator.py:21-241).
 *
 * The reference constructs one annotator per alt allele and calls one method
 * (vcf_parser.py:225-231), so the binding's own cost is the call's cost: a ctypes
 * call with nine converted arguments plus json.loads of the display text took
 * longer than the reference's whole Python method.  Here the allele strings are
 * read in place (compact ASCII str data, no encode), the entry is called through
 * the function pointer libavdb_hip.so exports (handed over by init(), so this
 * module links against nothing but Python), and the display dict is built
 * directly in the reference's key order.  All record arithmetic stays in the
 * library (K2's infer_end, K5a's display_shape / texts).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <string.h>

#include "avdb.h"

typedef int (*annotate_fn)(const void*, const uint8_t*, uint32_t, uint32_t, uint32_t, int, avdb_annotation*,
                           char*, size_t);

static annotate_fn g_fn = NULL;
static const void* g_ctx = NULL;

static PyObject *k_ls, *k_le, *k_nmid, *k_vc, *k_vca, *k_da, *k_sa;
static PyObject *vc_name[8], *vc_abbrev[8];

/* ASCII bytes of a str (in place) or bytes; -1 with ValueError for anything else */
static int ascii_view(PyObject* s, const char** p, Py_ssize_t* n) {
  if (PyUnicode_Check(s)) {
    if (PyUnicode_READY(s) < 0) return -1;
    if (!PyUnicode_IS_ASCII(s)) {
      PyErr_SetString(PyExc_ValueError, "non-ASCII allele: outside the kernels' byte-level contract");
      return -1;
    }
    *p = (const char*)PyUnicode_DATA(s);
    *n = PyUnicode_GET_LENGTH(s);
    return 0;
  }
  if (PyBytes_Check(s)) {
    *p = PyBytes_AS_STRING(s);
    *n = PyBytes_GET_SIZE(s);
    for (Py_ssize_t i = 0; i < *n; ++i)
      if ((*p)[i] & 0x80) {
        PyErr_SetString(PyExc_ValueError, "non-ASCII allele: outside the kernels' byte-level contract");
        return -1;
      }
    return 0;
  }
  PyErr_SetString(PyExc_TypeError, "alleles must be str or bytes");
  return -1;
}

/* ref + alt contiguous (the entry reads alt at offset len(ref)) and one K8a call */
static int annotate(PyObject* ref, PyObject* alt, uint32_t pos, int want, avdb_annotation* out, char* text,
                    size_t cap) {
  const char *rp, *ap;
  Py_ssize_t rn, an;
  if (!g_fn) {
    PyErr_SetString(PyExc_RuntimeError, "avdb_percall.init() not called");
    return -1;
  }
  if (ascii_view(ref, &rp, &rn) < 0 || ascii_view(alt, &ap, &an) < 0) return -1;
  if ((uint64_t)rn + (uint64_t)an > 0xFFFFFFFFull) {
    PyErr_SetString(PyExc_ValueError, "alleles longer than 2^32 bytes");
    return -1;
  }
  char stack[512];
  char* buf = stack;
  if (rn + an > (Py_ssize_t)sizeof(stack)) {
    buf = (char*)PyMem_Malloc((size_t)(rn + an));
    if (!buf) {
      PyErr_NoMemory();
      return -1;
    }
  }
  memcpy(buf, rp, (size_t)rn);
  memcpy(buf + rn, ap, (size_t)an);
  const int rc = g_fn(g_ctx, (const uint8_t*)buf, (uint32_t)rn, (uint32_t)an, pos, want, out, text, cap);
  if (buf != stack) PyMem_Free(buf);
  return rc;
}

static PyObject* py_init(PyObject* self, PyObject* args) {
  unsigned long long fn, ctx;
  if (!PyArg_ParseTuple(args, "KK", &fn, &ctx)) return NULL;
  g_fn = (annotate_fn)(uintptr_t)fn;
  g_ctx = (const void*)(uintptr_t)ctx;
  Py_RETURN_NONE;
}

/* end_lcp(ref, alt) -> (end - position, common-prefix length) */
static PyObject* py_end_lcp(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "end_lcp(ref, alt)");
    return NULL;
  }
  avdb_annotation out;
  const int rc = annotate(args[0], args[1], 0, 0, &out, NULL, 0);
  if (rc < 0) {
    if (!PyErr_Occurred()) PyErr_Format(PyExc_RuntimeError, "avdb_annotate_host failed (rc=%d)", rc);
    return NULL;
  }
  return Py_BuildValue("(iI)", out.end_rel, out.lcp);
}

static PyObject* text_obj(const char* p, Py_ssize_t n) { return PyUnicode_DecodeASCII(p, n, NULL); }

static int set_new(PyObject* d, PyObject* k, PyObject* v) {
  if (!v) return -1;
  const int rc = PyDict_SetItem(d, k, v);
  Py_DECREF(v);
  return rc;
}

/* display(ref, alt, label, pos) -> (dict, end - pos, lcp), or (None, end - pos, lcp)
 * when the display fields are the caller's (state 1) */
static PyObject* py_display(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 4) {
    PyErr_SetString(PyExc_TypeError, "display(ref, alt, label, pos)");
    return NULL;
  }
  PyObject *ref = args[0], *alt = args[1], *label = args[2];
  const unsigned long long pos = PyLong_AsUnsignedLongLong(args[3]);
  if (PyErr_Occurred()) return NULL;
  if (pos > 0xFFFFFFFFull) {
    PyErr_SetString(PyExc_ValueError, "position outside the kernels' u32 coordinates");
    return NULL;
  }
  char small[1024];
  char* text = small;
  size_t cap = sizeof(small);
  avdb_annotation out;
  int rc = annotate(ref, alt, (uint32_t)pos, 1, &out, text, cap);
  if (rc == AVDB_ERANGE) {
    cap = (size_t)out.display_bytes + out.sequence_bytes;
    text = (char*)PyMem_Malloc(cap ? cap : 1);
    if (!text) return PyErr_NoMemory();
    rc = annotate(ref, alt, (uint32_t)pos, 1, &out, text, cap);
  }
  PyObject* d = NULL;
  if (rc != 0) {
    if (!PyErr_Occurred()) PyErr_Format(PyExc_RuntimeError, "avdb_annotate_host failed (rc=%d)", rc);
    goto done;
  }
  if (out.state != 0) {
    d = Py_BuildValue("(OiI)", Py_None, out.end_rel, out.lcp);
    goto done;
  }
  if (out.variant_class > AVDB_VC_DELETION) {
    PyErr_Format(PyExc_RuntimeError, "avdb_annotate_host: variant class %u", out.variant_class);
    goto done;
  }
  {
    PyObject* dict = PyDict_New();
    if (!dict) goto done;
    const int cls = (int)out.variant_class;
    const int order_b = cls >= AVDB_VC_INDEL && cls <= AVDB_VC_DUPLICATION;
    int bad = set_new(dict, k_ls, PyLong_FromUnsignedLong(out.location_start)) ||
              set_new(dict, k_le, PyLong_FromUnsignedLong(out.location_end));
    const int snv = cls == AVDB_VC_SNV;
    if (!bad && !snv && out.lcp > 0) {
      /* ':'.join((xstr(chrom), xstr(position), normRef, normAlt)) with '-' for an
       * empty normalized allele (:150,159-161) */
      const char *rp, *ap;
      Py_ssize_t rn, an;
      ascii_view(ref, &rp, &rn);
      ascii_view(alt, &ap, &an);
      const Py_ssize_t nrn = rn - (Py_ssize_t)out.lcp, nan_ = an - (Py_ssize_t)out.lcp;
      char sbuf[512];
      const size_t need = 24 + (size_t)(nrn > 0 ? nrn : 1) + (size_t)(nan_ > 0 ? nan_ : 1);
      char* t = need <= sizeof(sbuf) ? sbuf : (char*)PyMem_Malloc(need);
      PyObject* nm = NULL;
      if (t) {
        int k = snprintf(t, 24, ":%llu:", pos);
        if (nrn > 0) { memcpy(t + k, rp + out.lcp, (size_t)nrn); k += (int)nrn; } else t[k++] = '-';
        t[k++] = ':';
        if (nan_ > 0) { memcpy(t + k, ap + out.lcp, (size_t)nan_); k += (int)nan_; } else t[k++] = '-';
        PyObject* tail = text_obj(t, k);
        if (tail) {
          nm = PyUnicode_Concat(label, tail);
          Py_DECREF(tail);
        }
        if (t != sbuf) PyMem_Free(t);
      } else {
        PyErr_NoMemory();
      }
      bad = set_new(dict, k_nmid, nm);
    }
    PyObject* da = text_obj(text, out.display_bytes);
    PyObject* sa = text_obj(text + out.display_bytes, out.sequence_bytes);
    if (!bad && !order_b)
      bad = PyDict_SetItem(dict, k_vc, vc_name[cls]) || PyDict_SetItem(dict, k_vca, vc_abbrev[cls]);
    if (!bad) {
      bad = set_new(dict, k_da, da);
      da = NULL;
    }
    if (!bad) {
      bad = set_new(dict, k_sa, sa);
      sa = NULL;
    }
    Py_XDECREF(da);
    Py_XDECREF(sa);
    if (!bad && order_b)
      bad = PyDict_SetItem(dict, k_vc, vc_name[cls]) || PyDict_SetItem(dict, k_vca, vc_abbrev[cls]);
    if (bad) {
      Py_DECREF(dict);
      goto done;
    }
    d = Py_BuildValue("(NiI)", dict, out.end_rel, out.lcp);
  }
done:
  if (text != small) PyMem_Free(text);
  return d;
}

static PyMethodDef methods[] = {
    {"init", py_init, METH_VARARGS, "init(avdb_annotate_host address, host context address)"},
    {"end_lcp", (PyCFunction)(void (*)(void))py_end_lcp, METH_FASTCALL, "end_lcp(ref, alt) -> (end - pos, lcp)"},
    {"display", (PyCFunction)(void (*)(void))py_display, METH_FASTCALL,
     "display(ref, alt, label, pos) -> (attributes dict | None, end - pos, lcp)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "avdb_percall", NULL, -1, methods};

PyMODINIT_FUNC PyInit_avdb_percall(void) {
  static const char* names[8] = {"single nucleotide variant", "inversion", "substitution", "indel", "indel",
                                 "insertion", "duplication", "deletion"};
  static const char* abbrevs[8] = {"SNV", "MNV", "MNV", "INDEL", "INDEL", "INS", "DUP", "DEL"};
  k_ls = PyUnicode_InternFromString("location_start");
  k_le = PyUnicode_InternFromString("location_end");
  k_nmid = PyUnicode_InternFromString("normalized_metaseq_id");
  k_vc = PyUnicode_InternFromString("variant_class");
  k_vca = PyUnicode_InternFromString("variant_class_abbrev");
  k_da = PyUnicode_InternFromString("display_allele");
  k_sa = PyUnicode_InternFromString("sequence_allele");
  for (int i = 0; i < 8; ++i) {
    vc_name[i] = PyUnicode_InternFromString(names[i]);
    vc_abbrev[i] = PyUnicode_InternFromString(abbrevs[i]);
  }
  return PyModule_Create(&module);
}
