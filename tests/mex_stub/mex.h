/* mex.h — a minimal stand-in for MATLAB's MEX / MX C API, test infrastructure only.
 *
 * MATLAB is not installed in this image, so matlab/mpct_mex.c is compiled against
 * this header and driven by tests/mex_stub/mex_driver.c, which builds MATLAB-shaped arguments
 * (column-major numeric arrays, struct arrays, char arrays, uint64 handles), calls mexFunction,
 * and prints the outputs.  Only the subset of the documented API that mpct_mex.c uses is declared,
 * with MATLAB's signatures, so the same source compiles with the real `mex`. */
#ifndef MPCT_MEX_STUB_H
#define MPCT_MEX_STUB_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef size_t mwSize;
typedef size_t mwIndex;
typedef struct mxArray_tag mxArray;

typedef enum {
  mxUNKNOWN_CLASS = 0,
  mxCELL_CLASS,
  mxSTRUCT_CLASS,
  mxLOGICAL_CLASS,
  mxCHAR_CLASS,
  mxVOID_CLASS,
  mxDOUBLE_CLASS,
  mxSINGLE_CLASS,
  mxINT8_CLASS,
  mxUINT8_CLASS,
  mxINT16_CLASS,
  mxUINT16_CLASS,
  mxINT32_CLASS,
  mxUINT32_CLASS,
  mxINT64_CLASS,
  mxUINT64_CLASS
} mxClassID;

typedef enum { mxREAL = 0, mxCOMPLEX } mxComplexity;

mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c);
mxArray* mxCreateNumericArray(mwSize ndim, const mwSize* dims, mxClassID cls, mxComplexity c);
mxArray* mxCreateString(const char* s);
mxArray* mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char** names);
void mxSetField(mxArray* s, mwIndex i, const char* name, mxArray* value);
mxArray* mxGetField(const mxArray* s, mwIndex i, const char* name);
void mxDestroyArray(mxArray* a);

double* mxGetPr(const mxArray* a);
void* mxGetData(const mxArray* a);
size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
mwSize mxGetNumberOfDimensions(const mxArray* a);
const mwSize* mxGetDimensions(const mxArray* a);
mxClassID mxGetClassID(const mxArray* a);
int mxIsDouble(const mxArray* a);
int mxIsNumeric(const mxArray* a);
int mxIsStruct(const mxArray* a);
int mxIsChar(const mxArray* a);
int mxIsEmpty(const mxArray* a);
int mxIsComplex(const mxArray* a);
int mxIsSparse(const mxArray* a);
double mxGetScalar(const mxArray* a);
int mxGetString(const mxArray* a, char* buf, mwSize buflen);

void* mxMalloc(size_t n);
void* mxCalloc(size_t n, size_t size);
void mxFree(void* p);

void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexAtExit(void (*fn)(void));
int mexPrintf(const char* fmt, ...);

/* the gateway the MEX file defines */
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

#ifdef __cplusplus
}
#endif
#endif
