// ldpc_mi355x.hpp -- header-only C++ adapter with the reference decoder's
// shape, over the C-ABI of ldpc_mi355x.h.
//
// A caller written against the reference (code/x86/main_p.cpp:377-396,485)
//
//     CDecoder *dec = CreateDecoder("OMS", "sse", "fixed", p_decoder,
//                                   vSAT_NEG_VAR, vSAT_POS_VAR, vSAT_NEG_MSG, vSAT_POS_MSG);
//     dec->decode(i_llr /* char[16*N] */, o_llr /* char[16*N] */, NOMBRE_ITERATIONS);
//
// switches by constructing ldpc_mi355x::CDecoder_OMS_fixed_MI355X (or calling
// ldpc_mi355x::CreateDecoder with arch "mi355x") with the code table; the
// decode() call, its frame-major int8 layout, 0/1 output and the
// setOffset / setFactor / setVarRange / setMsgRange configuration are the
// same (code/x86/CDecoder/template/CDecoder.h:28-40, CDecoder_fixed.h:30-44,
// OMS/CDecoder_OMS_fixed_SSE.h, NMS/CDecoder_NMS_fixed_SSE.h).  Errors throw
// ldpc_mi355x::Error instead of printf + exit(0).
#pragma once

#include <stdexcept>
#include <string>

#include "ldpc_mi355x.h"

namespace ldpc_mi355x {

struct Error : std::runtime_error {
    int status;
    Error(int s, const std::string &m) : std::runtime_error(m), status(s) {}
};

inline void check(int s)
{
    if (s != LDPC_OK) throw Error(s, std::string(ldpc_strerror(s)) + ": " + ldpc_last_error());
}

// Shared, immutable code table (replaces the compile-time PosNoeudsVariable).
class Code {
public:
    explicit Code(const char *path) { check(ldpc_code_load(path, &h_)); }
    Code(int n, int m, int n_groups, const int *deg, const int *cnt, const uint32_t *edge_var)
    {
        check(ldpc_code_create(n, m, n_groups, deg, cnt, edge_var, &h_));
    }
    ~Code() { ldpc_code_destroy(h_); }
    Code(const Code &) = delete;
    Code &operator=(const Code &) = delete;
    const ldpc_code *get() const { return h_; }
    int n() const
    {
        int n = 0;
        check(ldpc_code_info(h_, &n, nullptr, nullptr, nullptr, nullptr));
        return n;
    }

private:
    ldpc_code *h_ = nullptr;
};

// code/x86/CDecoder/template/CDecoder.h:28-40
class CDecoder {
public:
    CDecoder(const Code &code, int nb_frames = 16, int device = 0) : n_(code.n()), frames_(nb_frames)
    {
        check(ldpc_ctx_create(code.get(), device, nb_frames, &ctx_));
        ldpc_params_default(&p_);
    }
    virtual ~CDecoder() { ldpc_ctx_destroy(ctx_); }
    CDecoder(const CDecoder &) = delete;
    CDecoder &operator=(const CDecoder &) = delete;

    virtual void setSigmaChannel(float sigB) { sigB_ = sigB; }
    virtual void setNumberOfIterations(int v) { nb_iters_ = v; }
    // int8 LLRs, frame-major [nb_frames][N]; writes 0/1 per bit
    virtual void decode(char var_nodes[], char Rprime_fix[], int nombre_iterations)
    {
        check(ldpc_decode_i8(ctx_, reinterpret_cast<const int8_t *>(var_nodes), reinterpret_cast<uint8_t *>(Rprime_fix),
                             frames_, nombre_iterations, &p_));
    }
    // float LLRs: the layered float min-sum (the reference's fixed-point
    // decoders ignore this overload, CDecoder_fixed_SSE.cpp:35-40)
    virtual void decode(float var_nodes[], char Rprime_fix[], int nombre_iterations)
    {
        ldpc_params fp = p_;
        fp.algo = (p_.algo == LDPC_ALGO_NMS) ? LDPC_ALGO_NMS : LDPC_ALGO_MS;
        check(ldpc_decode_f32(ctx_, var_nodes, reinterpret_cast<uint8_t *>(Rprime_fix), frames_, nombre_iterations,
                              &fp));
    }
    ldpc_ctx *context() { return ctx_; }

protected:
    ldpc_ctx *ctx_ = nullptr;
    ldpc_params p_{};
    int n_, frames_;
    float sigB_ = 0.f;
    int nb_iters_ = 0;
};

// code/x86/CDecoder/template/CDecoder_fixed.h:30-44
class CDecoder_fixed : public CDecoder {
public:
    using CDecoder::CDecoder;
    virtual void setVarRange(int min, int max)
    {
        p_.var_min = min;
        p_.var_max = max;
    }
    virtual void setMsgRange(int min, int max)
    {
        p_.msg_min = min;
        p_.msg_max = max;
    }
};

// code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.h
class CDecoder_OMS_fixed_MI355X : public CDecoder_fixed {
public:
    CDecoder_OMS_fixed_MI355X(const Code &code, int nb_frames = 16, int device = 0)
        : CDecoder_fixed(code, nb_frames, device)
    {
        p_.algo = LDPC_ALGO_OMS;
    }
    void setOffset(int offset)
    {
        if (offset_set_) throw Error(LDPC_EINVAL, "Offset value was already configured");   // :104-112
        p_.offset = offset;
        offset_set_ = true;
    }

private:
    bool offset_set_ = false;
};

// code/x86/CDecoder/NMS/CDecoder_NMS_fixed_SSE.h
class CDecoder_NMS_fixed_MI355X : public CDecoder_fixed {
public:
    CDecoder_NMS_fixed_MI355X(const Code &code, int nb_frames = 16, int device = 0)
        : CDecoder_fixed(code, nb_frames, device)
    {
        p_.algo = LDPC_ALGO_NMS;
    }
    void setFactor(int f) { p_.factor = f; }
};

// code/x86/main_p.cpp:133-141
struct param_decoder {
    int nb_iters = 30;
    int nms_factor_fixed = 29;
    float nms_factor_float = 0.75f;
    int oms_offset_fixed = 1;
    float oms_offset_float = 0.15f;
};

// code/x86/CDecoder/DecoderLibrary.h:44-134
inline CDecoder_fixed *CreateDecoder(const std::string &type, const std::string &arch, const std::string &format,
                                     const param_decoder &p, int vMin, int vMax, int mMin, int mMax, const Code &code,
                                     int nb_frames = 16, int device = 0)
{
    if (format != "fixed" || (arch != "mi355x" && arch != "sse"))
        throw Error(LDPC_EUNSUPPORTED, "decoder unavailable: " + type + "/" + arch + "/" + format);
    CDecoder_fixed *d = nullptr;
    if (type == "OMS") {
        auto *o = new CDecoder_OMS_fixed_MI355X(code, nb_frames, device);
        o->setOffset(p.oms_offset_fixed);
        d = o;
    } else if (type == "NMS") {
        auto *o = new CDecoder_NMS_fixed_MI355X(code, nb_frames, device);
        o->setFactor(p.nms_factor_fixed);
        d = o;
    } else {
        throw Error(LDPC_EUNSUPPORTED, "Requested LDPC decoder does not exist (" + arch + ":" + type + ")");
    }
    d->setVarRange(vMin, vMax);
    d->setMsgRange(mMin, mMax);
    return d;
}

}  // namespace ldpc_mi355x
