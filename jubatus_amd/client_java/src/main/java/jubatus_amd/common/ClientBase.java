// Common part of the generated Java clients (jenerator -l java).
//
// Reference: jubatus/client/common/client.hpp:29-85 (get_config, save, load,
// get_status, do_mix, get_proxy_status; every call sends the cluster name
// first). Transport: msgpack-rpc-java (org.msgpack.rpc.Client); results are
// converted with msgpack-java templates chosen by the generated code.
package jubatus_amd.common;

import java.net.UnknownHostException;
import java.util.Map;

import org.msgpack.MessagePack;
import org.msgpack.rpc.Client;
import org.msgpack.rpc.loop.EventLoop;
import org.msgpack.template.Template;
import org.msgpack.template.Templates;
import org.msgpack.type.Value;

public class ClientBase {
  protected final Client client;
  protected final MessagePack msgpack;
  protected String name;

  public ClientBase(String host, int port, String name, int timeoutSec) {
    try {
      EventLoop loop = EventLoop.defaultEventLoop();
      this.client = new Client(host, port, loop);
    } catch (UnknownHostException e) {
      throw new IllegalArgumentException(e);
    }
    this.client.setRequestTimeout(timeoutSec);
    this.msgpack = new MessagePack();
    this.name = name;
  }

  public String getName() {
    return name;
  }

  public void setName(String name) {
    this.name = name;
  }

  public Client getClient() {
    return client;
  }

  public void close() {
    client.close();
  }

  protected <T> Template<T> template(Class<T> c) {
    return msgpack.lookup(c);
  }

  protected <T> T call(String method, Template<T> ret, Object... args) {
    Object[] full = new Object[args.length + 1];
    full[0] = name;
    System.arraycopy(args, 0, full, 1, args.length);
    Value v = client.callApply(method, full);
    try {
      return msgpack.convert(v, ret);
    } catch (java.io.IOException e) {
      throw new RuntimeException(method + ": unexpected result type", e);
    }
  }

  public String getConfig() {
    return call("get_config", Templates.TString);
  }

  public Map<String, String> save(String id) {
    return call("save", Templates.tMap(Templates.TString, Templates.TString), id);
  }

  public Boolean load(String id) {
    return call("load", Templates.TBoolean, id);
  }

  public Map<String, Map<String, String>> getStatus() {
    return call("get_status",
        Templates.tMap(Templates.TString, Templates.tMap(Templates.TString, Templates.TString)));
  }

  public Boolean doMix() {
    return call("do_mix", Templates.TBoolean);
  }

  public Map<String, Map<String, String>> getProxyStatus() {
    return call("get_proxy_status",
        Templates.tMap(Templates.TString, Templates.tMap(Templates.TString, Templates.TString)));
  }
}
