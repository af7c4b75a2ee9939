/* fv_converter plug-in ABI (C, stable across compilers).
 *
 * Reference: jubatus/server/fv_converter/so_factory.cpp:41-106 and
 * dynamic_loader.cpp:44-94 - a config type with "method": "dynamic",
 * "path": <shared object>, "function": <factory symbol> plus free-form
 * string parameters. The reference ABI is C++ (`T* create(const
 * std::map<std::string, std::string>&)` returning a jubatus_core class);
 * ours is plain C so plug-ins build with any toolchain and load through
 * ctypes: the factory gets the parameters as parallel key/value arrays and
 * returns a jb_plugin whose `kind` says which one operation it implements.
 * Every plug-in library also exports `const char* version(void)`, logged
 * at load time as the reference does.
 */
#ifndef JB_PLUGIN_H_
#define JB_PLUGIN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JB_PLUGIN_ABI 1

enum jb_plugin_kind {
  JB_STRING_FEATURE = 1,     /* splitter: text -> tokens */
  JB_STRING_FILTER = 2,      /* text -> text */
  JB_NUM_FEATURE = 3,        /* (key, x) -> named values */
  JB_NUM_FILTER = 4,         /* x -> x' */
  JB_BINARY_FEATURE = 5,     /* (key, bytes) -> named values */
  JB_COMBINATION_FEATURE = 6 /* (left, right) -> value */
};

/* one token of a string feature: text[begin, begin+length) unless `value`
 * is non-NULL (then value[0, value_len)); `score` multiplies its weight */
typedef struct jb_token {
  int64_t begin, length;
  const char* value;
  int64_t value_len;
  double score;
} jb_token;

/* one named value (names stay valid until the next call on the plug-in) */
typedef struct jb_named {
  const char* name;
  double value;
} jb_named;

typedef struct jb_plugin {
  int abi;  /* JB_PLUGIN_ABI */
  int kind; /* jb_plugin_kind */
  void* self;
  /* return the number of outputs; when it exceeds `cap` the caller retries
   * with a bigger buffer (outputs beyond cap are not written) */
  int (*string_feature)(void* self, const char* text, int64_t len, jb_token* out, int cap);
  /* returns the output length; when it exceeds `cap` the caller retries */
  int64_t (*string_filter)(void* self, const char* in, int64_t len, char* out, int64_t cap);
  int (*num_feature)(void* self, const char* key, double x, jb_named* out, int cap);
  double (*num_filter)(void* self, double x);
  int (*binary_feature)(void* self, const char* key, const char* data, int64_t len, jb_named* out,
                        int cap);
  double (*combination)(void* self, double left, double right);
  void (*destroy)(void* self);
} jb_plugin;

typedef jb_plugin* (*jb_plugin_factory)(const char** keys, const char** values, int n);

#ifdef __cplusplus
}
#endif

#endif /* JB_PLUGIN_H_ */
