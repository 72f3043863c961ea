/* mex_driver.c — test infrastructure: a minimal implementation of the MX / MEX API declared in
 * tests/mex_stub/mex.h plus a driver that plays MATLAB's part for matlab/mpct_mex.c.
 *
 * Input (stdin): a sequence of calls
 *     CALL <nlhs> <nrhs>   then nrhs argument specs
 * Spec grammar (whitespace-separated tokens, values column-major as MATLAB stores them):
 *     D <ndims> <dims...> <values...>      double array
 *     I <ndims> <dims...> <values...>      int32 array
 *     S <string>                           char row vector (no spaces)
 *     T <m> <n> <nfields> <names...>  then m*n*nfields specs (element-major, fields in order)
 *     P <call> <k>                         output k of an earlier call (handles)
 * Output (stdout): for each call "CALL <i> OK" and every output as "OUT <k> <spec>" (uint64 as
 * "U 2 1 1 <v>", doubles with %.17g, char arrays with space / percent as %20 / %25), or "CALL <i> ERR <id> <message>" when mexFunction raised
 * (mexErrMsgIdAndTxt longjmps back here, as MATLAB unwinds).  mxMalloc'd memory is released after
 * every call, as MATLAB does.  At EOF the registered mexAtExit function runs. */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

struct mxArray_tag {
  mxClassID cls;
  mwSize ndim;
  mwSize dims[4];
  void* data;       /* numeric / char payload */
  int nfields;
  char** names;
  mxArray** fields; /* [nelem * nfields] */
};

static size_t nelem(const mxArray* a) {
  size_t n = 1;
  for (mwSize k = 0; k < a->ndim; ++k) n *= a->dims[k];
  return n;
}

static size_t esize(mxClassID c) {
  switch (c) {
    case mxDOUBLE_CLASS: case mxINT64_CLASS: case mxUINT64_CLASS: return 8;
    case mxSINGLE_CLASS: case mxINT32_CLASS: case mxUINT32_CLASS: return 4;
    case mxCHAR_CLASS: case mxINT16_CLASS: case mxUINT16_CLASS: return 2;
    default: return 1;
  }
}

/* ---- mxMalloc bookkeeping: freed after each mexFunction call */
static void** g_allocs;
static size_t g_nalloc, g_capalloc;

void* mxMalloc(size_t n) {
  void* p = malloc(n ? n : 1);
  if (g_nalloc == g_capalloc) {
    g_capalloc = g_capalloc ? 2 * g_capalloc : 256;
    g_allocs = (void**)realloc(g_allocs, g_capalloc * sizeof(void*));
  }
  g_allocs[g_nalloc++] = p;
  return p;
}
void* mxCalloc(size_t n, size_t size) {
  void* p = mxMalloc(n * size);
  memset(p, 0, (n && size) ? n * size : 1);
  return p;
}
void mxFree(void* p) {
  for (size_t k = 0; k < g_nalloc; ++k)
    if (g_allocs[k] == p) {
      free(p);
      g_allocs[k] = g_allocs[--g_nalloc];
      return;
    }
}
static void free_call_allocs(void) {
  for (size_t k = 0; k < g_nalloc; ++k) free(g_allocs[k]);
  g_nalloc = 0;
}

/* ---- arrays */
mxArray* mxCreateNumericArray(mwSize ndim, const mwSize* dims, mxClassID cls, mxComplexity c) {
  (void)c;
  mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
  a->cls = cls;
  a->ndim = ndim < 2 ? 2 : ndim;
  a->dims[0] = a->dims[1] = 1;
  for (mwSize k = 0; k < ndim; ++k) a->dims[k] = dims[k];
  a->data = calloc(nelem(a) ? nelem(a) : 1, esize(cls));
  return a;
}
mxArray* mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c) {
  mwSize d[2] = {m, n};
  return mxCreateNumericArray(2, d, cls, c);
}
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) { return mxCreateNumericMatrix(m, n, mxDOUBLE_CLASS, c); }
mxArray* mxCreateDoubleScalar(double v) {
  mxArray* a = mxCreateDoubleMatrix(1, 1, mxREAL);
  *(double*)a->data = v;
  return a;
}
mxArray* mxCreateString(const char* s) {
  const size_t n = strlen(s);
  mxArray* a = mxCreateNumericMatrix(1, n, mxCHAR_CLASS, mxREAL);
  for (size_t k = 0; k < n; ++k) ((uint16_t*)a->data)[k] = (uint16_t)(unsigned char)s[k];
  return a;
}
mxArray* mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char** names) {
  mxArray* a = mxCreateNumericMatrix(m, n, mxSTRUCT_CLASS, mxREAL);
  a->nfields = nfields;
  a->names = (char**)calloc((size_t)nfields, sizeof(char*));
  for (int f = 0; f < nfields; ++f) a->names[f] = strdup(names[f]);
  a->fields = (mxArray**)calloc(nelem(a) * (size_t)nfields + 1, sizeof(mxArray*));
  return a;
}
static int field_index(const mxArray* s, const char* name) {
  for (int f = 0; f < s->nfields; ++f)
    if (!strcmp(s->names[f], name)) return f;
  return -1;
}
void mxSetField(mxArray* s, mwIndex i, const char* name, mxArray* v) {
  const int f = field_index(s, name);
  if (f >= 0) s->fields[i * (size_t)s->nfields + f] = v;
}
mxArray* mxGetField(const mxArray* s, mwIndex i, const char* name) {
  if (!s || s->cls != mxSTRUCT_CLASS || i >= nelem(s)) return NULL;
  const int f = field_index(s, name);
  return f < 0 ? NULL : s->fields[i * (size_t)s->nfields + f];
}
void mxDestroyArray(mxArray* a) {
  if (!a) return;
  if (a->cls == mxSTRUCT_CLASS) {
    for (size_t k = 0; k < nelem(a) * (size_t)a->nfields; ++k) mxDestroyArray(a->fields[k]);
    for (int f = 0; f < a->nfields; ++f) free(a->names[f]);
    free(a->names);
    free(a->fields);
  }
  free(a->data);
  free(a);
}
double* mxGetPr(const mxArray* a) { return a->cls == mxDOUBLE_CLASS ? (double*)a->data : NULL; }
void* mxGetData(const mxArray* a) { return a->data; }
size_t mxGetM(const mxArray* a) { return a->dims[0]; }
size_t mxGetN(const mxArray* a) {
  size_t n = 1;
  for (mwSize k = 1; k < a->ndim; ++k) n *= a->dims[k];
  return n;
}
size_t mxGetNumberOfElements(const mxArray* a) { return nelem(a); }
mwSize mxGetNumberOfDimensions(const mxArray* a) { return a->ndim; }
const mwSize* mxGetDimensions(const mxArray* a) { return a->dims; }
mxClassID mxGetClassID(const mxArray* a) { return a->cls; }
int mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
int mxIsNumeric(const mxArray* a) { return a->cls >= mxDOUBLE_CLASS; }
int mxIsStruct(const mxArray* a) { return a->cls == mxSTRUCT_CLASS; }
int mxIsChar(const mxArray* a) { return a->cls == mxCHAR_CLASS; }
int mxIsEmpty(const mxArray* a) { return nelem(a) == 0; }
int mxIsComplex(const mxArray* a) { (void)a; return 0; }
int mxIsSparse(const mxArray* a) { (void)a; return 0; }
double mxGetScalar(const mxArray* a) {
  if (nelem(a) == 0) return 0.0;
  switch (a->cls) {
    case mxDOUBLE_CLASS: return *(double*)a->data;
    case mxINT32_CLASS: return *(int32_t*)a->data;
    case mxUINT64_CLASS: return (double)*(uint64_t*)a->data;
    case mxINT64_CLASS: return (double)*(int64_t*)a->data;
    default: return 0.0;
  }
}
int mxGetString(const mxArray* a, char* buf, mwSize len) {
  if (a->cls != mxCHAR_CLASS || len == 0) return 1;
  const size_t n = nelem(a);
  size_t k = 0;
  for (; k < n && k + 1 < len; ++k) buf[k] = (char)((uint16_t*)a->data)[k];
  buf[k] = 0;
  return k < n ? 1 : 0;
}

/* ---- mex */
static jmp_buf g_jmp;
static char g_errid[128], g_errmsg[1024];
static void (*g_atexit)(void);

void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_errmsg, sizeof g_errmsg, fmt, ap);
  va_end(ap);
  snprintf(g_errid, sizeof g_errid, "%s", id);
  longjmp(g_jmp, 1);
}
int mexAtExit(void (*fn)(void)) {
  g_atexit = fn;
  return 0;
}
int mexPrintf(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  const int n = vfprintf(stderr, fmt, ap);
  va_end(ap);
  return n;
}

/* ---- the driver */
#define MAXCALLS 64
static mxArray* g_out[MAXCALLS][16];

static char* tok(void) {
  static char buf[4096];
  if (scanf("%4095s", buf) != 1) {
    fprintf(stderr, "driver: unexpected end of input\n");
    exit(3);
  }
  return buf;
}

static mxArray* parse(void) {
  const char* t = tok();
  if (!strcmp(t, "D") || !strcmp(t, "I")) {
    const int dbl = t[0] == 'D';
    mwSize dims[4] = {0, 0, 1, 1};
    const int nd = atoi(tok());
    for (int k = 0; k < nd; ++k) dims[k] = (mwSize)atol(tok());
    mxArray* a = mxCreateNumericArray((mwSize)nd, dims, dbl ? mxDOUBLE_CLASS : mxINT32_CLASS, mxREAL);
    for (size_t k = 0; k < nelem(a); ++k) {
      if (dbl) ((double*)a->data)[k] = strtod(tok(), NULL);
      else ((int32_t*)a->data)[k] = (int32_t)atol(tok());
    }
    return a;
  }
  if (!strcmp(t, "S")) return mxCreateString(tok());
  if (!strcmp(t, "P")) {
    const int c = atoi(tok()), k = atoi(tok());
    const mxArray* o = g_out[c][k];
    mxArray* a = mxCreateNumericArray(o->ndim, o->dims, o->cls, mxREAL);
    memcpy(a->data, o->data, nelem(o) * esize(o->cls));
    return a;
  }
  if (!strcmp(t, "T")) {
    const mwSize m = (mwSize)atol(tok()), n = (mwSize)atol(tok());
    const int nf = atoi(tok());
    char** names = (char**)calloc((size_t)nf, sizeof(char*));
    for (int f = 0; f < nf; ++f) names[f] = strdup(tok());
    mxArray* a = mxCreateStructMatrix(m, n, nf, (const char**)names);
    for (size_t e = 0; e < (size_t)m * n; ++e)
      for (int f = 0; f < nf; ++f) a->fields[e * (size_t)nf + f] = parse();
    for (int f = 0; f < nf; ++f) free(names[f]);
    free(names);
    return a;
  }
  fprintf(stderr, "driver: bad spec token '%s'\n", t);
  exit(3);
}

static void print(const mxArray* a) {
  if (a->cls == mxCHAR_CLASS) {
    printf("S ");
    for (size_t k = 0; k < nelem(a); ++k) {
      const char ch = (char)((uint16_t*)a->data)[k];
      if (ch == ' ') fputs("%20", stdout);
      else if (ch == '%') fputs("%25", stdout);
      else putchar(ch);
    }
    printf("\n");
    return;
  }
  const char* c = a->cls == mxDOUBLE_CLASS ? "D" : a->cls == mxUINT64_CLASS ? "U" : "I";
  printf("%s %d", c, (int)a->ndim);
  for (mwSize k = 0; k < a->ndim; ++k) printf(" %zu", a->dims[k]);
  for (size_t k = 0; k < nelem(a); ++k) {
    if (a->cls == mxDOUBLE_CLASS) printf(" %.17g", ((double*)a->data)[k]);
    else if (a->cls == mxUINT64_CLASS) printf(" %llu", (unsigned long long)((uint64_t*)a->data)[k]);
    else printf(" %d", ((int32_t*)a->data)[k]);
  }
  printf("\n");
}

int main(void) {
  char word[16];
  int call = 0;
  while (scanf("%15s", word) == 1) {
    if (strcmp(word, "CALL")) {
      fprintf(stderr, "driver: expected CALL, got '%s'\n", word);
      return 3;
    }
    if (call >= MAXCALLS) return 3;
    const int nlhs = atoi(tok()), nrhs = atoi(tok());
    mxArray* prhs[16] = {0};
    mxArray* plhs[16] = {0};
    for (int k = 0; k < nrhs && k < 16; ++k) prhs[k] = parse();
    if (setjmp(g_jmp) == 0) {
      mexFunction(nlhs, plhs, nrhs, (const mxArray**)prhs);
      printf("CALL %d OK\n", call);
      for (int k = 0; k < 16; ++k)
        if (plhs[k]) {
          printf("OUT %d ", k);
          print(plhs[k]);
          g_out[call][k] = plhs[k];
        }
    } else {
      for (char* p = g_errmsg; *p; ++p)
        if (*p == '\n') *p = ' ';
      printf("CALL %d ERR %s %s\n", call, g_errid, g_errmsg);
    }
    fflush(stdout);
    free_call_allocs();
    for (int k = 0; k < nrhs && k < 16; ++k) mxDestroyArray(prhs[k]);
    ++call;
  }
  if (g_atexit) g_atexit();
  return 0;
}
