/*
 * cfg.c — encoder.cfg handling, restating JM 8.6 configfile.c › Configure / ParseCommand /
 * GetConfigFileContent / ParseContent / ParameterNameToMapIndex / PatchInp [J].
 * "Key = Value" lines, '#' comments, quoted strings; -d <default.cfg>, -f <extra.cfg>,
 * -p Key=Value overrides applied in command-line order; unknown keys are an error.
 * Keys follow JM 8.6 spellings; JM>=10 spellings are accepted as aliases.
 */
#include <ctype.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "jmhost.h"

typedef struct {
    const char *name;
    int type;          /* 0 int, 1 string */
    size_t off;
    int lo, hi;
} map_entry;

#define OFF(f) offsetof(jm_input, f)
static const map_entry Map[] = {
    {"InputFile", 1, OFF(infile), 0, 0},
    {"OutputFile", 1, OFF(outfile), 0, 0},
    {"ReconFile", 1, OFF(reconfile), 0, 0},
    {"FramesToBeEncoded", 0, OFF(frames), 1, 1 << 20},
    {"StartFrame", 0, OFF(start_frame), 0, 1 << 20},
    {"SourceWidth", 0, OFF(width), 16, 8192},
    {"SourceHeight", 0, OFF(height), 16, 8192},
    {"IntraPeriod", 0, OFF(intra_period), 0, 1 << 20},
    {"QPFirstFrame", 0, OFF(qp_i), 0, 51},
    {"QPISlice", 0, OFF(qp_i), 0, 51},
    {"QPRemainingFrame", 0, OFF(qp_p), 0, 51},
    {"QPPSlice", 0, OFF(qp_p), 0, 51},
    {"SearchRange", 0, OFF(search_range), 1, 64},
    {"SearchMode", 0, OFF(search_mode), -1, 3},
    {"UseFME", 0, OFF(search_mode), 0, 3},
    {"UseHadamard", 0, OFF(use_hadamard), 0, 1},
    {"NumberReferenceFrames", 0, OFF(num_ref_frames), 1, 16},
    {"RestrictSearchRange", 0, OFF(restrict_search_range), 0, 2},
    {"InterSearch16x16", 0, OFF(inter_search[1]), 0, 1},
    {"InterSearch16x8", 0, OFF(inter_search[2]), 0, 1},
    {"InterSearch8x16", 0, OFF(inter_search[3]), 0, 1},
    {"InterSearch8x8", 0, OFF(inter_search[4]), 0, 1},
    {"InterSearch8x4", 0, OFF(inter_search[5]), 0, 1},
    {"InterSearch4x8", 0, OFF(inter_search[6]), 0, 1},
    {"InterSearch4x4", 0, OFF(inter_search[7]), 0, 1},
    {"RDOptimization", 0, OFF(rdopt), 0, 2},
    {"ProfileIDC", 0, OFF(profile_idc), 66, 144},
    {"Transform8x8Mode", 0, OFF(transform_8x8_mode), 0, 2},
    {"LevelIDC", 0, OFF(level_idc), 9, 62},
    {"SymbolMode", 0, OFF(symbol_mode), 0, 1},
    {"ContextInitMethod", 0, OFF(context_init_method), 0, 1},
    {"SourceBitDepthLuma", 0, OFF(bit_depth_luma), 8, 14},
    {"SourceBitDepthChroma", 0, OFF(bit_depth_chroma), 8, 14},
    {"FixedModelNumber", 0, OFF(model_number), 0, 2},
    {"LoopFilterParametersFlag", 0, OFF(lf_params_flag), 0, 1},
    {"LoopFilterDisable", 0, OFF(lf_disable), 0, 1},
    {"LoopFilterAlphaC0Offset", 0, OFF(lf_alpha), -6, 6},
    {"LoopFilterBetaOffset", 0, OFF(lf_beta), -6, 6},
    {"ChromaQPOffset", 0, OFF(chroma_qp_offset), -12, 12},
    {"UseConstrainedIntraPred", 0, OFF(constrained_intra), 0, 1},
    {"FrameRate", 0, OFF(frame_rate), 1, 1000},
    {"HIPDevice", 0, OFF(hip_device), 0, 63},
    {"PipelineDepth", 0, OFF(pipeline_depth), 0, 20},
    {"JMCallSurface", 0, OFF(jm_call_surface), 0, 1},
    {"WriterThreads", 0, OFF(writer_threads), 0, 64},
    {"JMVersion", 0, OFF(jm_version), 8, 99},
    {"QOffsetIntra", 0, OFF(qoff_intra), -1, JMH_QOFFSET_MAX},
    {"QOffsetInter", 0, OFF(qoff_inter), -1, JMH_QOFFSET_MAX},
    {"AdaptiveRounding", 0, OFF(adaptive_rounding), 0, 1},
    {"OffsetMatrixPresentFlag", 0, OFF(offset_matrix_present), 0, 1},
    {"EPZSDualRefinement", 0, OFF(epzs_dual), 0, 4},
    {"SliceMode", 0, OFF(slice_mode), 0, 3},
    {"SliceArgument", 0, OFF(slice_arg), 1, 1 << 20},
    {"EPZSSubPelME", 0, OFF(epzs_subpel), 0, 1},
    {"EPZSSubPelThresScale", 0, OFF(epzs_subpel_thres), 0, JMH_EPZS_SCALE_MAX},
    {"EPZSMinThresScale", 0, OFF(epzs_min_thres), 0, JMH_EPZS_SCALE_MAX},
    {"EPZSMaxThresScale", 0, OFF(epzs_max_thres), 0, JMH_EPZS_SCALE_MAX},
    {NULL, 0, 0, 0, 0}};
#undef OFF

void jm_input_defaults(jm_input *inp) {
    memset(inp, 0, sizeof(*inp));
    strcpy(inp->infile, "synthetic:0");
    strcpy(inp->outfile, "test.264");
    inp->frames = 3;
    inp->width = 176; inp->height = 144;
    inp->intra_period = 0;
    inp->qp_i = 28; inp->qp_p = 28;
    inp->search_range = 16;
    inp->search_mode = 0;
    inp->use_hadamard = 1;
    inp->num_ref_frames = 1;
    inp->restrict_search_range = 2;
    for (int i = 1; i <= 7; i++) inp->inter_search[i] = 1;
    inp->profile_idc = 66;
    inp->level_idc = 40;
    inp->frame_rate = 30;
    inp->writer_threads = 4;
    inp->jm_version = 8;
    inp->qoff_intra = inp->qoff_inter = -1;
    inp->slice_arg = 50;                       /* encoder.cfg SliceArgument default [J] */
    inp->bit_depth_luma = inp->bit_depth_chroma = 8;
}

int jm_set_param(jm_input *inp, const char *key, const char *val, char *err, int errlen) {
    for (const map_entry *m = Map; m->name; m++) {
        if (strcmp(m->name, key)) continue;
        char *base = (char *)inp + m->off;
        if (m->type == 1) {
            snprintf(base, 512, "%s", val);
            return 0;
        }
        char *end;
        long v = strtol(val, &end, 10);
        if (end == val || *end) {
            snprintf(err, errlen, "Parsing error in config: '%s' expects an integer, got '%s'", key, val);
            return -1;
        }
        if (!strcmp(key, "UseFME")) v = v == 0 ? 0 : 1;   /* JM 8.6 UseFME 0 == fast full search */
        if (v < m->lo || v > m->hi) {
            snprintf(err, errlen, "Error in input parameter %s: value %ld out of range [%d,%d]", key, v, m->lo, m->hi);
            return -1;
        }
        *(int *)base = (int)v;
        return 0;
    }
    snprintf(err, errlen, "Parameter Name '%s' not recognized.", key);
    return -1;
}

/* ParseContent [J]: tokenise "Key = Value" pairs, '#' to end of line is a comment */
int jm_parse_content(jm_input *inp, const char *buf, char *err, int errlen) {
    const char *p = buf;
    while (*p) {
        while (*p && (isspace((unsigned char)*p))) p++;
        if (!*p) break;
        if (*p == '#') { while (*p && *p != '\n') p++; continue; }
        char key[128], val[512];
        int k = 0;
        while (*p && !isspace((unsigned char)*p) && *p != '=' && *p != '#' && k < 127) key[k++] = *p++;
        key[k] = 0;
        while (*p == ' ' || *p == '\t') p++;
        if (*p != '=') {
            snprintf(err, errlen, "Parsing error in config file: '=' expected after '%s'", key);
            return -1;
        }
        p++;
        while (*p == ' ' || *p == '\t') p++;
        int v = 0;
        if (*p == '"') {
            p++;
            while (*p && *p != '"' && v < 511) val[v++] = *p++;
            if (*p == '"') p++;
        } else {
            while (*p && !isspace((unsigned char)*p) && *p != '#' && v < 511) val[v++] = *p++;
        }
        val[v] = 0;
        if (jm_set_param(inp, key, val, err, errlen)) return -1;
    }
    return 0;
}

static int parse_file(jm_input *inp, const char *fn, char *err, int errlen) {
    FILE *f = fopen(fn, "rb");
    if (!f) { snprintf(err, errlen, "Cannot open configuration file %s.", fn); return -1; }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = malloc(n + 1);
    long got = (long)fread(buf, 1, n, f);
    fclose(f);
    buf[got] = 0;
    int r = jm_parse_content(inp, buf, err, errlen);
    free(buf);
    return r;
}

int jm_patch_input(jm_input *inp, char *err, int errlen) {
    if (inp->rdopt > 1) { snprintf(err, errlen, "RDOptimization=%d not supported (0 or 1)", inp->rdopt); return -1; }
    if (inp->rdopt && inp->jm_call_surface) { snprintf(err, errlen, "JMCallSurface=1 checks the RDO-off decision (RDOptimization=0)"); return -1; }
    if (inp->symbol_mode && inp->profile_idc == 66) { snprintf(err, errlen, "SymbolMode=1 (CABAC) is not allowed in the Baseline profile (ProfileIDC=66)"); return -1; }
    if (inp->symbol_mode && inp->context_init_method) { snprintf(err, errlen, "ContextInitMethod=1 (adaptive CABAC model selection) not supported (0: FixedModelNumber)"); return -1; }
    if (inp->symbol_mode && inp->model_number) { snprintf(err, errlen, "FixedModelNumber=%d not supported (0: cabac_init_idc 0)", inp->model_number); return -1; }
    if (inp->search_mode != 0 && inp->search_mode != -1 && inp->search_mode != 3) { snprintf(err, errlen, "SearchMode=%d not supported (use -1, 0 or 3)", inp->search_mode); return -1; }
    if (inp->search_range > 32 && inp->search_mode != 3) { snprintf(err, errlen, "SearchRange=%d > 32 needs SearchMode=3 (the FFS / full-search windows are LDS-resident at 32)", inp->search_range); return -1; }
    if (inp->num_ref_frames != 1) { snprintf(err, errlen, "NumberReferenceFrames=%d not supported (1)", inp->num_ref_frames); return -1; }
    if (inp->profile_idc != 66 && inp->profile_idc != 77 && inp->profile_idc != 100 && inp->profile_idc != 110) { snprintf(err, errlen, "ProfileIDC=%d not supported (66, 77, 100 or 110)", inp->profile_idc); return -1; }
    if (inp->bit_depth_luma > 10 || inp->bit_depth_chroma != inp->bit_depth_luma) { snprintf(err, errlen, "SourceBitDepthLuma=%d / SourceBitDepthChroma=%d not supported (equal, 8..10)", inp->bit_depth_luma, inp->bit_depth_chroma); return -1; }
    if (inp->bit_depth_luma > 8 && inp->profile_idc != 110) { snprintf(err, errlen, "SourceBitDepthLuma=%d requires ProfileIDC=110 (High 10)", inp->bit_depth_luma); return -1; }
    if (inp->bit_depth_luma > 8 && inp->jm_call_surface) { snprintf(err, errlen, "JMCallSurface=1 runs the 8-bit per-block seams (SourceBitDepthLuma 8)"); return -1; }
    if (inp->transform_8x8_mode == 2) { snprintf(err, errlen, "Transform8x8Mode=2 not supported (0 or 1)"); return -1; }
    if (inp->transform_8x8_mode && inp->profile_idc < 100) { snprintf(err, errlen, "Transform8x8Mode=1 requires ProfileIDC=100 (High)"); return -1; }
    if ((inp->width & 1) || (inp->height & 1)) { snprintf(err, errlen, "Source size must be even"); return -1; }
    if (inp->jm_version == 9) { snprintf(err, errlen, "JMVersion=9 not supported (8 or >= 10)"); return -1; }
    if (inp->epzs_dual > 1) { snprintf(err, errlen, "EPZSDualRefinement=%d not supported (0 or 1)", inp->epzs_dual); return -1; }
    if (inp->slice_mode > 1) { snprintf(err, errlen, "SliceMode=%d not supported (0 or 1: SliceArgument macroblocks per slice)", inp->slice_mode); return -1; }
    if (inp->adaptive_rounding) { snprintf(err, errlen, "AdaptiveRounding=1 not supported (0)"); return -1; }
    if (inp->offset_matrix_present) { snprintf(err, errlen, "OffsetMatrixPresentFlag=1 not supported (flat lists: QOffsetIntra / QOffsetInter)"); return -1; }
    if (inp->jm_version < 10 && (inp->qoff_intra >= 0 || inp->qoff_inter >= 0)) { snprintf(err, errlen, "QOffsetIntra / QOffsetInter need JMVersion >= 10"); return -1; }
    if (inp->jm_version >= 10) {               /* q_offsets.c defaults (OffsetMatrixPresentFlag 0) [J] */
        if (inp->qoff_intra < 0) inp->qoff_intra = 682;
        if (inp->qoff_inter < 0) inp->qoff_inter = 342;
    }
    return 0;
}

int jm_configure(jm_input *inp, int argc, char **argv, char *err, int errlen) {
    int have_d = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-h")) {
            snprintf(err, errlen, "usage: lencod [-d default.cfg] [-f file.cfg] [-p Key=Value]...");
            return -1;
        } else if (!strcmp(argv[i], "-d") && i + 1 < argc) {
            if (parse_file(inp, argv[++i], err, errlen)) return -1;
            have_d = 1;
        } else if (!strcmp(argv[i], "-f") && i + 1 < argc) {
            if (parse_file(inp, argv[++i], err, errlen)) return -1;
        } else if (!strcmp(argv[i], "-p") && i + 1 < argc) {
            if (jm_parse_content(inp, argv[++i], err, errlen)) return -1;
        } else {
            snprintf(err, errlen, "Error in command line, ac %d, around string '%s', missing -f or -p parameters?", i, argv[i]);
            return -1;
        }
    }
    (void)have_d;
    return jm_patch_input(inp, err, errlen);
}

void jm_fill_config(const jm_input *inp, jmh_config *cfg) {
    memset(cfg, 0, sizeof(*cfg));
    cfg->width = (inp->width + 15) & ~15;
    cfg->height = (inp->height + 15) & ~15;
    cfg->search_range = inp->search_range;
    cfg->search_mode = inp->search_mode;
    cfg->use_hadamard = inp->use_hadamard;
    cfg->restrict_search_range = inp->restrict_search_range;
    for (int i = 1; i <= 7; i++) cfg->inter_search[i] = inp->inter_search[i];
    cfg->num_ref_frames = inp->num_ref_frames;
    cfg->constrained_intra_pred = inp->constrained_intra;
    cfg->num_frame_slots = 2;
    cfg->pipeline_depth = inp->pipeline_depth;
    cfg->transform_8x8_mode = inp->transform_8x8_mode;
    cfg->jm_version = inp->jm_version;
    cfg->epzs_dual_refinement = inp->epzs_dual;
    cfg->epzs_subpel_me = inp->epzs_subpel;
    cfg->epzs_subpel_thres_scale = inp->epzs_subpel_thres;
    cfg->epzs_min_thres_scale = inp->epzs_min_thres;
    cfg->epzs_max_thres_scale = inp->epzs_max_thres;
    cfg->slice_mbs = inp->slice_mode == 1 ? inp->slice_arg : 0;
    cfg->bit_depth = inp->bit_depth_luma;
    cfg->rdo = inp->rdopt;
    cfg->symbol_mode = inp->symbol_mode;
    if (inp->jm_version >= 10) { cfg->quant_offset[0] = inp->qoff_intra; cfg->quant_offset[1] = inp->qoff_inter; }
}
