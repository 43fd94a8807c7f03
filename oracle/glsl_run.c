/* oracle/glsl_run.c -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/glsl_run; never linked into
 * the product, never run on the GPU box).
 *
 * Runs the REFERENCE'S OWN shaders -- /root/reference/shaders/vertex_shader.glsl and
 * octree_fragment_shader.glsl, read from where they lie at run time, never copied -- through a
 * real GLSL 4.30 implementation: the image's Mesa 23.2 llvmpipe (swrast_dri.so, a software
 * OpenGL 4.5 core driver). There is no X server or EGL in the image, so this program is its
 * own minimal DRI "swrast" loader: it opens the driver, creates a screen, an OpenGL 4.3 core
 * context and a drawable through the driver's __DRI_CORE / __DRI_SWRAST extensions
 * (GL/internal/dri_interface.h), and reaches GL through libglapi's dispatch.
 *
 * The GL side restates what the reference's host does for one frame:
 *   - Raytracer::setupBuffers (src/raytracer.cpp:74-152): seven std430 SSBOs at bindings 0-6
 *     (centre+radius, material+albedo, fuzz+ri+0+0, node min+childrenOffset (as float),
 *     node max+objectsOffset (as float), object counts (int), object indices (int)) and the
 *     uniforms useOctree / octreeNodeCount / sphereCount / numSamples / maxDepth / iResolution;
 *   - the frame (src/raytracer.cpp:491-499): view, cameraPosition, cameraZoom, then
 *     glDrawArrays(GL_TRIANGLES, 0, 6) over the full-screen quad of Raytracer::setupQuad
 *     (src/raytracer.cpp:42-55; attribute 0 = position, 1 = texcoord, 5 floats a vertex).
 * It draws into a W x H GL_RGBA32F framebuffer object instead of the window (the reference
 * never reads pixels back) and reads FragColor back as float.
 *
 * usage: glsl_run SHADER_DIR INPUT OUTPUT [PRELUDE]
 *   PRELUDE (analysis only, tools/glsl_builtins_check.py): GLSL text inserted after the
 *   fragment shader's #version line, in memory (the reference's file is never changed) -- used
 *   to substitute the oracle's canonical builtins for llvmpipe's and so measure how much of
 *   the remaining difference is the builtins'.  Its leading lines of the form
 *   "//@replace OLD<TAB>NEW" each replace the one occurrence of OLD in the fragment shader (in
 *   memory, before the insertion; OLD must occur exactly once) -- the canonical prelude uses one
 *   to read the pixel centre from gl_FragCoord instead of the interpolated FragCoord varying.
 *   INPUT (little endian): int32 W, H, numSamples, maxDepth, useOctree, nSpheres, nNodes,
 *   nIndices; float32 view[16] (column-major, as glUniformMatrix4fv takes glm), cameraPosition[3],
 *   cameraZoom; then float32[nSpheres*4] x3, float32[nNodes*4] x2, int32[nNodes],
 *   int32[nIndices].  OUTPUT: float32[H][W][4], GL row order (row 0 = bottom).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <GL/gl.h>
#include <GL/glext.h>
#include <GL/internal/dri_interface.h>

#ifndef DRI_DRIVER_PATH
#define DRI_DRIVER_PATH "/usr/lib/x86_64-linux-gnu/dri/swrast_dri.so"
#endif

static int g_w = 1, g_h = 1;

static void die(const char *m) {
    fprintf(stderr, "glsl_run: %s\n", m);
    exit(2);
}

/* the swrast loader: a drawable of the frame's size; nothing is ever presented */
static void get_drawable_info(__DRIdrawable *d, int *x, int *y, int *w, int *h, void *lp) {
    (void)d;
    (void)lp;
    *x = 0;
    *y = 0;
    *w = g_w;
    *h = g_h;
}
static void put_image(__DRIdrawable *d, int op, int x, int y, int w, int h, char *data, void *lp) {
    (void)d; (void)op; (void)x; (void)y; (void)w; (void)h; (void)data; (void)lp;
}
static void get_image(__DRIdrawable *d, int x, int y, int w, int h, char *data, void *lp) {
    (void)d; (void)x; (void)y; (void)lp;
    memset(data, 0, (size_t)w * (size_t)h * 4);
}
static const __DRIswrastLoaderExtension k_loader = {
    {__DRI_SWRAST_LOADER, 1}, get_drawable_info, put_image, get_image, NULL, NULL, NULL, NULL, NULL, NULL};
static const __DRIextension *k_loader_exts[] = {&k_loader.base, NULL};

/* GL entry points through libglapi (the driver installs its dispatch table on bindContext) */
typedef void *(*get_proc_fn)(const char *);
static get_proc_fn g_get_proc;
static void *gp(const char *name) {
    void *f = g_get_proc(name);
    if (!f) {
        fprintf(stderr, "glsl_run: no GL entry point %s\n", name);
        exit(2);
    }
    return f;
}
#define GLF(type, name) type name = (type)gp(#name)
/* GL 1.x entry points have no PFN typedefs in glext.h */
typedef const GLubyte *(*PFNGLGETSTRINGPROC)(GLenum);
typedef GLenum (*PFNGLGETERRORPROC)(void);
typedef void (*PFNGLVIEWPORTPROC)(GLint, GLint, GLsizei, GLsizei);
typedef void (*PFNGLCLEARCOLORPROC)(GLfloat, GLfloat, GLfloat, GLfloat);
typedef void (*PFNGLCLEARPROC)(GLbitfield);
typedef void (*PFNGLDRAWARRAYSPROC)(GLenum, GLint, GLsizei);
typedef void (*PFNGLFINISHPROC)(void);
typedef void (*PFNGLREADBUFFERPROC)(GLenum);
typedef void (*PFNGLPIXELSTOREIPROC)(GLenum, GLint);
typedef void (*PFNGLREADPIXELSPROC)(GLint, GLint, GLsizei, GLsizei, GLenum, GLenum, void *);
typedef void (*PFNGLGENTEXTURESPROC)(GLsizei, GLuint *);
typedef void (*PFNGLBINDTEXTUREPROC)(GLenum, GLuint);
typedef void (*PFNGLTEXIMAGE2DPROC)(GLenum, GLint, GLint, GLsizei, GLsizei, GLint, GLenum, GLenum, const void *);
typedef void (*PFNGLTEXPARAMETERIPROC)(GLenum, GLenum, GLint);

static char *read_file(const char *path, size_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *b = (char *)malloc((size_t)len + 1);
    if (!b || fread(b, 1, (size_t)len, f) != (size_t)len) die("read failed");
    b[len] = 0;
    fclose(f);
    if (n) *n = (size_t)len;
    return b;
}

int main(int argc, char **argv) {
    if (argc != 4 && argc != 5) die("usage: glsl_run SHADER_DIR INPUT OUTPUT [PRELUDE]");
    size_t in_n = 0;
    char *in = read_file(argv[2], &in_n);
    if (!in || in_n < 8 * 4 + 20 * 4) die("bad input file");
    const int32_t *hd = (const int32_t *)in;
    const int W = hd[0], H = hd[1], ns = hd[2], md = hd[3], use_octree = hd[4], nS = hd[5], nN = hd[6], nI = hd[7];
    const float *view = (const float *)(in + 32), *pos = view + 16, *zoom = pos + 3;
    const char *p = (const char *)(zoom + 1);
    const size_t need = 32 + 80 + (size_t)nS * 48 + (size_t)nN * 36 + (size_t)nI * 4;
    if (W <= 0 || H <= 0 || nS <= 0 || nN < 0 || nI < 0 || in_n != need) die("input size does not match its header");
    const float *sph_cr = (const float *)p, *sph_ma = sph_cr + 4 * (size_t)nS, *sph_fr = sph_ma + 4 * (size_t)nS;
    const float *nd_min = sph_fr + 4 * (size_t)nS, *nd_max = nd_min + 4 * (size_t)nN;
    const int32_t *nd_cnt = (const int32_t *)(nd_max + 4 * (size_t)nN), *idx = nd_cnt + nN;
    g_w = W;
    g_h = H;

    char path[4096];
    snprintf(path, sizeof path, "%s/vertex_shader.glsl", argv[1]);
    char *vs_src = read_file(path, NULL);
    snprintf(path, sizeof path, "%s/octree_fragment_shader.glsl", argv[1]);
    char *fs_src = read_file(path, NULL);
    if (argc == 5 && fs_src) {  /* the prelude goes right after the #version line */
        char *pre = read_file(argv[4], NULL);
        if (!pre) die("cannot read the prelude");
        while (strncmp(pre, "//@replace ", 11) == 0) {  /* its replacement lines */
            char *eol = strchr(pre, '\n'), *tab = strchr(pre + 11, '\t');
            if (!eol || !tab || tab > eol) die("bad //@replace line");
            *eol = 0;
            *tab = 0;
            const char *old = pre + 11, *rep = tab + 1;
            char *at = strstr(fs_src, old);
            if (!at || strstr(at + 1, old)) die("//@replace: OLD must occur exactly once in the fragment shader");
            const size_t a = (size_t)(at - fs_src), lo = strlen(old), lr = strlen(rep), c = strlen(at + lo);
            char *m = (char *)malloc(a + lr + c + 1);
            if (!m) die("out of memory");
            memcpy(m, fs_src, a);
            memcpy(m + a, rep, lr);
            memcpy(m + a + lr, at + lo, c + 1);
            fs_src = m;
            pre = eol + 1;
        }
        char *nl = strchr(fs_src, '\n');
        if (!pre || !nl || strncmp(fs_src, "#version", 8) != 0) die("cannot insert the prelude");
        const size_t a = (size_t)(nl + 1 - fs_src), b = strlen(pre), c = strlen(nl + 1);
        char *m = (char *)malloc(a + b + c + 1);
        if (!m) die("out of memory");
        memcpy(m, fs_src, a);
        memcpy(m + a, pre, b);
        memcpy(m + a + b, nl + 1, c + 1);
        fs_src = m;
    }
    if (!vs_src || !fs_src) die("cannot read the reference shaders");

    /* the driver and its loader-facing extensions */
    void *glapi = dlopen("libglapi.so.0", RTLD_NOW | RTLD_GLOBAL);
    if (!glapi) die(dlerror());
    g_get_proc = (get_proc_fn)dlsym(glapi, "_glapi_get_proc_address");
    void *drv = dlopen(DRI_DRIVER_PATH, RTLD_NOW | RTLD_GLOBAL);
    if (!drv || !g_get_proc) die(dlerror());
    const __DRIextension **(*get_ext)(void) =
        (const __DRIextension **(*)(void))dlsym(drv, "__driDriverGetExtensions_swrast");
    if (!get_ext) die("no __driDriverGetExtensions_swrast");
    const __DRIextension **ext = get_ext();
    const __DRIcoreExtension *core = NULL;
    const __DRIswrastExtension *sw = NULL;
    for (int i = 0; ext[i]; ++i) {
        if (!strcmp(ext[i]->name, __DRI_CORE)) core = (const __DRIcoreExtension *)ext[i];
        if (!strcmp(ext[i]->name, __DRI_SWRAST)) sw = (const __DRIswrastExtension *)ext[i];
    }
    if (!core || !sw || sw->base.version < 4) die("driver lacks DRI core / swrast v4");
    const __DRIconfig **configs = NULL;
    __DRIscreen *scr = sw->createNewScreen2(0, k_loader_exts, ext, &configs, NULL);
    if (!scr || !configs || !configs[0]) die("createNewScreen2 failed");
    const uint32_t attribs[] = {__DRI_CTX_ATTRIB_MAJOR_VERSION, 4, __DRI_CTX_ATTRIB_MINOR_VERSION, 3};
    unsigned err = 0;
    __DRIcontext *ctx = sw->createContextAttribs(scr, __DRI_API_OPENGL_CORE, configs[0], NULL, 2, attribs, &err, NULL);
    if (!ctx) die("createContextAttribs (OpenGL 4.3 core) failed");
    __DRIdrawable *dr = sw->createNewDrawable(scr, configs[0], NULL);
    if (!dr || !core->bindContext(ctx, dr, dr)) die("bindContext failed");

    GLF(PFNGLGETSTRINGPROC, glGetString);
    GLF(PFNGLGETERRORPROC, glGetError);
    GLF(PFNGLCREATESHADERPROC, glCreateShader);
    GLF(PFNGLSHADERSOURCEPROC, glShaderSource);
    GLF(PFNGLCOMPILESHADERPROC, glCompileShader);
    GLF(PFNGLGETSHADERIVPROC, glGetShaderiv);
    GLF(PFNGLGETSHADERINFOLOGPROC, glGetShaderInfoLog);
    GLF(PFNGLCREATEPROGRAMPROC, glCreateProgram);
    GLF(PFNGLATTACHSHADERPROC, glAttachShader);
    GLF(PFNGLLINKPROGRAMPROC, glLinkProgram);
    GLF(PFNGLGETPROGRAMIVPROC, glGetProgramiv);
    GLF(PFNGLGETPROGRAMINFOLOGPROC, glGetProgramInfoLog);
    GLF(PFNGLUSEPROGRAMPROC, glUseProgram);
    GLF(PFNGLGETUNIFORMLOCATIONPROC, glGetUniformLocation);
    GLF(PFNGLUNIFORM1IPROC, glUniform1i);
    GLF(PFNGLUNIFORM1FPROC, glUniform1f);
    GLF(PFNGLUNIFORM3FPROC, glUniform3f);
    GLF(PFNGLUNIFORMMATRIX4FVPROC, glUniformMatrix4fv);
    GLF(PFNGLGENBUFFERSPROC, glGenBuffers);
    GLF(PFNGLBINDBUFFERPROC, glBindBuffer);
    GLF(PFNGLBUFFERDATAPROC, glBufferData);
    GLF(PFNGLBINDBUFFERBASEPROC, glBindBufferBase);
    GLF(PFNGLGENVERTEXARRAYSPROC, glGenVertexArrays);
    GLF(PFNGLBINDVERTEXARRAYPROC, glBindVertexArray);
    GLF(PFNGLVERTEXATTRIBPOINTERPROC, glVertexAttribPointer);
    GLF(PFNGLENABLEVERTEXATTRIBARRAYPROC, glEnableVertexAttribArray);
    GLF(PFNGLGENTEXTURESPROC, glGenTextures);
    GLF(PFNGLBINDTEXTUREPROC, glBindTexture);
    GLF(PFNGLTEXIMAGE2DPROC, glTexImage2D);
    GLF(PFNGLTEXPARAMETERIPROC, glTexParameteri);
    GLF(PFNGLGENFRAMEBUFFERSPROC, glGenFramebuffers);
    GLF(PFNGLBINDFRAMEBUFFERPROC, glBindFramebuffer);
    GLF(PFNGLFRAMEBUFFERTEXTURE2DPROC, glFramebufferTexture2D);
    GLF(PFNGLCHECKFRAMEBUFFERSTATUSPROC, glCheckFramebufferStatus);
    GLF(PFNGLDRAWBUFFERSPROC, glDrawBuffers);
    GLF(PFNGLVIEWPORTPROC, glViewport);
    GLF(PFNGLCLEARCOLORPROC, glClearColor);
    GLF(PFNGLCLEARPROC, glClear);
    GLF(PFNGLDRAWARRAYSPROC, glDrawArrays);
    GLF(PFNGLFINISHPROC, glFinish);
    GLF(PFNGLREADBUFFERPROC, glReadBuffer);
    GLF(PFNGLPIXELSTOREIPROC, glPixelStorei);
    GLF(PFNGLREADPIXELSPROC, glReadPixels);
    GLF(PFNGLGETINTEGER64VPROC, glGetInteger64v);
    fprintf(stderr, "glsl_run: %s / %s\n", (const char *)glGetString(GL_RENDERER), (const char *)glGetString(GL_VERSION));
    /* (llvmpipe reports a 128 MiB GL_MAX_SHADER_STORAGE_BLOCK_SIZE but reads larger buffers whole:
     * the C3 node arrays, 175 MB each, give frames bit-identical to the oracle's) */
    GLint64 max_ssbo = 0;
    glGetInteger64v(GL_MAX_SHADER_STORAGE_BLOCK_SIZE, &max_ssbo);
    fprintf(stderr, "glsl_run: GL_MAX_SHADER_STORAGE_BLOCK_SIZE %lld\n", (long long)max_ssbo);

    /* the reference's program */
    GLuint sh[2];
    const char *srcs[2] = {vs_src, fs_src};
    const GLenum kinds[2] = {GL_VERTEX_SHADER, GL_FRAGMENT_SHADER};
    GLuint prog = glCreateProgram();
    for (int i = 0; i < 2; ++i) {
        sh[i] = glCreateShader(kinds[i]);
        glShaderSource(sh[i], 1, &srcs[i], NULL);
        glCompileShader(sh[i]);
        GLint ok = 0;
        glGetShaderiv(sh[i], GL_COMPILE_STATUS, &ok);
        if (!ok) {
            char log[8192];
            glGetShaderInfoLog(sh[i], sizeof log, NULL, log);
            fprintf(stderr, "%s\n", log);
            die("shader compile failed");
        }
        glAttachShader(prog, sh[i]);
    }
    glLinkProgram(prog);
    GLint linked = 0;
    glGetProgramiv(prog, GL_LINK_STATUS, &linked);
    if (!linked) {
        char log[8192];
        glGetProgramInfoLog(prog, sizeof log, NULL, log);
        fprintf(stderr, "%s\n", log);
        die("program link failed");
    }

    /* the float framebuffer the frame is drawn into */
    GLuint tex, fbo;
    glGenTextures(1, &tex);
    glBindTexture(GL_TEXTURE_2D, tex);
    glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA32F, W, H, 0, GL_RGBA, GL_FLOAT, NULL);
    glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, GL_NEAREST);
    glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, GL_NEAREST);
    glGenFramebuffers(1, &fbo);
    glBindFramebuffer(GL_FRAMEBUFFER, fbo);
    glFramebufferTexture2D(GL_FRAMEBUFFER, GL_COLOR_ATTACHMENT0, GL_TEXTURE_2D, tex, 0);
    const GLenum db = GL_COLOR_ATTACHMENT0;
    glDrawBuffers(1, &db);
    if (glCheckFramebufferStatus(GL_FRAMEBUFFER) != GL_FRAMEBUFFER_COMPLETE) die("framebuffer incomplete");
    glViewport(0, 0, W, H);

    /* setupBuffers: the seven SSBOs (childrenOffset / objectsOffset travel as floats, as the
     * reference's glm::vec4(node.min, node.childrenOffset) makes them) */
    const void *data[7] = {sph_cr, sph_ma, sph_fr, nd_min, nd_max, nd_cnt, idx};
    const size_t bytes[7] = {16 * (size_t)nS, 16 * (size_t)nS, 16 * (size_t)nS, 16 * (size_t)nN, 16 * (size_t)nN,
                             4 * (size_t)nN, 4 * (size_t)nI};
    GLuint ssbo[7];
    glGenBuffers(7, ssbo);
    for (int b = 0; b < 7; ++b) {
        glBindBuffer(GL_SHADER_STORAGE_BUFFER, ssbo[b]);
        glBufferData(GL_SHADER_STORAGE_BUFFER, (GLsizeiptr)(bytes[b] ? bytes[b] : 4), bytes[b] ? data[b] : NULL,
                     GL_STATIC_DRAW);
        glBindBufferBase(GL_SHADER_STORAGE_BUFFER, (GLuint)b, ssbo[b]);
    }
    glUseProgram(prog);
    glUniform1i(glGetUniformLocation(prog, "useOctree"), use_octree);
    glUniform1i(glGetUniformLocation(prog, "octreeNodeCount"), nN);
    glUniform1i(glGetUniformLocation(prog, "sphereCount"), nS);
    glUniform1i(glGetUniformLocation(prog, "numSamples"), ns);
    glUniform1i(glGetUniformLocation(prog, "maxDepth"), md);
    glUniform3f(glGetUniformLocation(prog, "iResolution"), (float)W, (float)H, 0.0f);
    glUniformMatrix4fv(glGetUniformLocation(prog, "view"), 1, GL_FALSE, view);
    glUniform3f(glGetUniformLocation(prog, "cameraPosition"), pos[0], pos[1], pos[2]);
    glUniform1f(glGetUniformLocation(prog, "cameraZoom"), zoom[0]);

    /* the full-screen quad: two triangles, position xyz + texcoord uv per vertex */
    static const float quad[30] = {-1, 1, 0, 0, 1, -1, -1, 0, 0, 0, 1, -1, 0, 1, 0,
                                   -1, 1, 0, 0, 1, 1,  -1, 0, 1, 0, 1, 1,  0, 1, 1};
    GLuint vao, vbo;
    glGenVertexArrays(1, &vao);
    glBindVertexArray(vao);
    glGenBuffers(1, &vbo);
    glBindBuffer(GL_ARRAY_BUFFER, vbo);
    glBufferData(GL_ARRAY_BUFFER, sizeof quad, quad, GL_STATIC_DRAW);
    glVertexAttribPointer(0, 3, GL_FLOAT, GL_FALSE, 5 * sizeof(float), (void *)0);
    glEnableVertexAttribArray(0);
    glVertexAttribPointer(1, 2, GL_FLOAT, GL_FALSE, 5 * sizeof(float), (void *)(3 * sizeof(float)));
    glEnableVertexAttribArray(1);

    glClearColor(0.2f, 0.2f, 0.2f, 1.0f);
    glClear(GL_COLOR_BUFFER_BIT);
    struct timespec t0, t1;
    glFinish();
    clock_gettime(CLOCK_MONOTONIC, &t0);
    glDrawArrays(GL_TRIANGLES, 0, 6);
    glFinish();
    clock_gettime(CLOCK_MONOTONIC, &t1);
    fprintf(stderr, "glsl_run: draw %.1f ms\n", (double)(t1.tv_sec - t0.tv_sec) * 1e3 + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-6);
    float *out = (float *)malloc((size_t)W * (size_t)H * 16);
    if (!out) die("out of memory");
    glReadBuffer(GL_COLOR_ATTACHMENT0);
    glPixelStorei(GL_PACK_ALIGNMENT, 4);
    glReadPixels(0, 0, W, H, GL_RGBA, GL_FLOAT, out);
    const GLenum e = glGetError();
    if (e != GL_NO_ERROR) {
        fprintf(stderr, "glsl_run: GL error 0x%x\n", (unsigned)e);
        return 2;
    }
    FILE *f = fopen(argv[3], "wb");
    if (!f || fwrite(out, 16, (size_t)W * (size_t)H, f) != (size_t)W * (size_t)H) die("cannot write the output");
    fclose(f);
    core->unbindContext(ctx);
    return 0;
}
